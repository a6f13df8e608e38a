#!/bin/bash
# Parallel graph-cut labeling with cells strided over the parts: graph-cut /
# end-to-end correspondence tests, then the H and F wall time to 0.99 (LO
# lists = the labeling) at GCR_GC_PARTS = 64 / 256 / 1024.
set -u
O=gpurun_out/gcparts
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_graphcut.py tests/test_gpu_graphcut.py tests/test_homography.py tests/test_fundamental.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for g in 64 256 1024; do
  for w in h f; do
    GCR_GC_PARTS=$g timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 0 --no-hbm-probe > $O/${w}_p$g.log 2>&1 || { tail -20 $O/${w}_p$g.log; exit 1; }
  done
done
echo "session done"
