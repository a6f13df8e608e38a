#!/bin/bash
# k_score_fm A/B: parity, M2 bench (L2 re-read vs lane permute), F, H
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_fm.log 2>&1
rc=$?; tail -3 gpurun_out/tests_fm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 0 --no-hbm-probe > gpurun_out/bench_m2.log 2>&1 || exit 1
GCR_PROBE=32 timeout -k 10 300 python bench.py --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/bench_m2_shfl.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/bench_f.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/bench_h.log 2>&1 || exit 1
echo done
