#!/bin/bash
# round-4 session 29: k_lo_fold value reads issued with the counts -- fold
# tests, latency A/B against the previous build (separate processes, interleaved)
set -u
O=gpurun_out/r4_s29; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_refit_reuse.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
timeout -k 10 200 python -u tools/lat_ab.py --workload m2 --reps 4 new: > $O/lat_new$i.log 2>&1 || { tail -20 $O/lat_new$i.log; exit 1; }
GCR_LIB=libgcr_base.so timeout -k 10 200 python -u tools/lat_ab.py --workload m2 --reps 4 base: > $O/lat_base$i.log 2>&1 || { tail -20 $O/lat_base$i.log; exit 1; }
done
grep -h "median" $O/lat_*.log | cut -c1-120
