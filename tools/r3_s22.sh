#!/bin/bash
# fold cycle counts, fold + summary tests, latency A/B wide vs one-lane fold
set -u
D=gpurun_out/r3_s22
mkdir -p $D
timeout -k 10 120 python -u tools/fold_bench.py > $D/fold_bench.log 2>&1 || { echo "fold bench failed"; tail -5 $D/fold_bench.log; exit 1; }
cat $D/fold_bench.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_summary.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $D/tests.log
[ $rc -eq 0 ] || exit $rc
for w in m2 m1; do timeout -k 10 300 python -u tools/lat_ab.py --workload $w --reps 4 seq: wide:GCR_LO_FOLD=wide > $D/lat_$w.log 2>&1 || { echo "lat $w failed"; tail -5 $D/lat_$w.log; exit 1; }; tail -2 $D/lat_$w.log; done
