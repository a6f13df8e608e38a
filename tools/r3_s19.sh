#!/bin/bash
# Wide exact LO fold: device fold tests, the full GPU suite, latency A/B
# (wide vs one-lane fold), default bench line, rocprofv3 + PMC for M2.
set -u
T=${TAG:-r3_s19}
D=gpurun_out/$T
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py -x -q --timeout 120 --timeout-method thread > $D/fold_tests.log 2>&1; rc=$?
echo "fold tests rc=$rc"; tail -3 $D/fold_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $D/tests.log
[ $rc -eq 0 ] || exit $rc
for w in m2 m1 h; do timeout -k 10 300 python -u tools/lat_ab.py --workload $w --reps 3 wide: seq:GCR_LO_FOLD=seq > $D/lat_$w.log 2>&1 || { echo "lat $w failed"; tail -5 $D/lat_$w.log; exit 1; }; tail -4 $D/lat_$w.log; done
timeout -k 10 300 python -u tools/lat_ab.py --workload f --reps 2 wide: seq:GCR_LO_FOLD=seq > $D/lat_f.log 2>&1 || { echo "lat f failed"; exit 1; }
tail -4 $D/lat_f.log
timeout -k 10 400 python bench.py > $D/bench.log 2> $D/bench.err || { echo "bench failed"; tail -5 $D/bench.err; exit 1; }
tail -c 400 $D/bench.log; echo
WL=m2 TAG=$T/m2 STATS=1 PMC=1 bash tools/r3_measure.sh || exit 1
echo "session $T done"
