#!/bin/bash
# chained fused launches: bench-config parity first, then the full suite, the
# driver-shaped line chained / unchained
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_config.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_chain.log 2>&1
rc=$?; tail -3 gpurun_out/tests_chain.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_all.log 2>&1
rc=$?; tail -3 gpurun_out/tests_all.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > gpurun_out/chain_on_$rep.log 2>&1 || exit 1
  GCR_VERIFY_CHAIN=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > gpurun_out/chain_off_$rep.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --gpus 1 --steps 2000 --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > gpurun_out/chain_on_2000.log 2>&1 || exit 1
echo done
