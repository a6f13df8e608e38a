#!/bin/bash
# k_score_fm VALU breakdown: SQ pass per GCR_PROBE setting (results invalid
# under a probe; only the counters and kernel time are read)
set -u
mkdir -p gpurun_out
for p in 0 1 2 4 8 6; do
  GCR_PROBE=$p PMC_DIR=gpurun_out/probe_$p PMC_FILE=tools/pmc_sets_p1.txt BENCH_ARGS="--steps 20 --warmup 2 --cpu-seconds 0 --no-latency --no-hbm-probe" bash tools/pmc_session.sh > gpurun_out/probe_$p.log 2>&1 || { echo "probe $p failed"; exit 1; }
  GCR_PROBE=$p timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > gpurun_out/probe_bench_$p.log 2>&1 || exit 1
done
echo done
