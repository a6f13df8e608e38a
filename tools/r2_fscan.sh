#!/bin/bash
# F verify with the compaction scan inside the scorer
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_fscan.log 2>&1
rc=$?; tail -3 gpurun_out/tests_fscan.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/fscan_$rep.log 2>&1 || exit 1
done
echo done
