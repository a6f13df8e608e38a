#!/bin/bash
# k_score_fm session: parity of the scorers, M2 bench line, SQ counter pass
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_fm.log 2>&1
rc=$?; tail -5 gpurun_out/tests_fm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 0 --no-hbm-probe > gpurun_out/bench_m2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/bench_f.log 2>&1 || exit 1
PMC_DIR=gpurun_out/pmc_m2 PMC_FILE=tools/pmc_sets_sq.txt BENCH_ARGS="--steps 20 --warmup 2 --cpu-seconds 0 --no-latency --no-hbm-probe" bash tools/pmc_session.sh
