#!/bin/bash
# Homography generator lanes per slot with deferred selection (fixed groups):
# H line at GCR_GEN_G = 4 / 8 / 16 / 32.
set -u
O=gpurun_out/hg
mkdir -p $O
for g in 4 8 16 32; do
  GCR_GEN_G=$g timeout -k 10 300 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe --no-latency > $O/h_g$g.log 2>&1 || { tail -20 $O/h_g$g.log; exit 1; }
done
echo "session done"
