#!/bin/bash
# experiment: fused feature-major scorer at 8 hypotheses per workgroup (two per CU)
set -u
mkdir -p gpurun_out
GCR_FM_H=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_config.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "fused or chained" > gpurun_out/tests_h8.log 2>&1
rc=$?; tail -3 gpurun_out/tests_h8.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  GCR_FM_H=8 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > gpurun_out/h8_$rep.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > gpurun_out/h16_$rep.log 2>&1 || exit 1
done
echo done
