#!/bin/bash
# correspondence scorers held to 64 VGPRs (dynamic LDS): parity, then F / H
# lines with the two-stream pipeline on and off
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_geo64.log 2>&1
rc=$?; tail -3 gpurun_out/tests_geo64.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for w in f h; do
  timeout -k 10 300 python bench.py --workload $w --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/g64_${w}_$rep.log 2>&1 || exit 1
  GCR_VERIFY_PIPE=0 timeout -k 10 300 python bench.py --workload $w --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/g64_${w}_nopipe_$rep.log 2>&1 || exit 1
done
done
echo done
