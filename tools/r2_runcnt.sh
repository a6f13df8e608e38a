#!/bin/bash
# Exact-pass inlier counts: one LDS atomic per run of equal hypotheses in a
# batch (default) vs one per inlier lane (GCR_PROBE=256).  Parity tests, then
# the M2 (20 / 2000 steps), M1, H and F lines both ways.
set -u
O=gpurun_out/runcnt
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for pr in 0 256; do
  GCR_PROBE=$pr timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-hbm-probe --no-latency > $O/m2_20_p$pr.log 2>&1 || { tail -20 $O/m2_20_p$pr.log; exit 1; }
  GCR_PROBE=$pr timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 50 --cpu-seconds 0 --no-hbm-probe --no-latency > $O/m2_2000_p$pr.log 2>&1 || { tail -20 $O/m2_2000_p$pr.log; exit 1; }
  for w in m1 h f; do
    GCR_PROBE=$pr timeout -k 10 200 python bench.py --workload $w --cpu-seconds 0 --no-hbm-probe --no-latency > $O/${w}_p$pr.log 2>&1 || { tail -20 $O/${w}_p$pr.log; exit 1; }
  done
done
echo "session done"
