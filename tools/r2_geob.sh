#!/bin/bash
# geo band loop variant: parity of the correspondence suites, F / H lines
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_geo_band.py tests/test_fundamental.py tests/test_homography.py tests/test_gpu_bench_config.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "not fused and not chained" > gpurun_out/tests_geob.log 2>&1
rc=$?; tail -2 gpurun_out/tests_geob.log; [ $rc -eq 0 ] || exit $rc
for w in f h; do
  timeout -k 10 300 python bench.py --workload $w --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/gb_${w}.log 2>&1 || exit 1
  GCR_VERIFY_PIPE=0 timeout -k 10 300 python bench.py --workload $w --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/gb_${w}_nopipe.log 2>&1 || exit 1
done
echo done
