#!/bin/bash
# A/B of GCR_PROBE variants on the M2 bench line (same box, interleaved)
set -u
mkdir -p gpurun_out
for rep in 1 2; do
for p in ${PROBES:-0 64}; do
  GCR_PROBE=$p timeout -k 10 120 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-latency --no-hbm-probe ${BENCH_ARGS:-} > gpurun_out/ab_${p}_$rep.log 2>&1 || exit 1
done
done
echo done
