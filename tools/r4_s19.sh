#!/bin/bash
# round-4 session 18: branch-free run walk -- fold tests, fold bench, M2 latency
set -u
O=gpurun_out/r4_s19; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -u tools/fold_bench.py > $O/fold_bench.log 2>&1 || { cat $O/fold_bench.log; exit 1; }
cat $O/fold_bench.log
timeout -k 10 300 python -u tools/lat_ab.py --workload m2 --reps 5 base: seq:GCR_LO_FOLD=seq > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
cat $O/lat.log
