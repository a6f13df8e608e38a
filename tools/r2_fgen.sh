#!/bin/bash
# F generator session: parity, bench line, SQ counter passes on the F bench
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fundamental.py tests/test_gpu_geo_band.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_f.log 2>&1 || { tail -30 gpurun_out/tests_f.log; exit 1; }
tail -3 gpurun_out/tests_f.log
timeout -k 10 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/benchf.log 2>&1 || exit 1
PMC_DIR=gpurun_out/pmc_f PMC_FILE=tools/pmc_sets_sq.txt BENCH_ARGS="--workload f --steps 20 --warmup 2 --cpu-seconds 0 --no-latency --no-hbm-probe" bash tools/pmc_session.sh
