#!/bin/bash
# skeleton timing of k_score_fm under GCR_PROBE combinations (invalid results)
set -u
mkdir -p gpurun_out
for p in 4 5 12 13; do
  GCR_PROBE=$p timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > gpurun_out/probe_bench_$p.log 2>&1 || exit 1
done
echo done
