#!/bin/bash
# round-4 session 11: three-chain fold -- device fold tests, small-scorer
# parity, fold stamps, latency A/B of the block fold vs the one-lane fold
set -u
O=gpurun_out/r4_s11; mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_fold.py -x -q --timeout 120 --timeout-method thread > $O/fold_tests.log 2>&1 || { tail -30 $O/fold_tests.log; exit 1; }
tail -2 $O/fold_tests.log
timeout -k 10 120 python -u tools/lo_stamp_probe.py --models 2 > $O/stamps.log 2>&1 || { cat $O/stamps.log; exit 1; }
cat $O/stamps.log
timeout -k 10 300 python -u tools/lat_ab.py --workload m2 --reps 5 base: seq:GCR_LO_FOLD=seq > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
cat $O/lat.log
