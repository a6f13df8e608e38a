#!/bin/bash
# F generator lanes per slot under the two-stream pipeline
set -u
mkdir -p gpurun_out
for g in 8 16 32 64; do
  GCR_GEN_G=$g timeout -k 10 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/fg_$g.log 2>&1 || exit 1
done
echo done
