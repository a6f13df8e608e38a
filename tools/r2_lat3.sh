#!/bin/bash
# end-to-end parity suites + the latency leg
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_all.log 2>&1
rc=$?; tail -3 gpurun_out/tests_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/bench_drv.log 2>&1 || exit 1
echo done
