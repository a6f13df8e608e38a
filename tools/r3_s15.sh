#!/bin/bash
set -u
D=gpurun_out/${TAG:-r3_s15}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $D/tests.log
[ $rc -eq 0 ] || exit $rc
GCR_ZEROCOPY=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_summary.py tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > $D/tests_nozc.log 2>&1; rc=$?; echo "tests nozc rc=$rc"; tail -1 $D/tests_nozc.log
[ $rc -eq 0 ] || exit $rc
for w in m2 h; do timeout -k 10 300 python -u tools/lat_ab.py --workload $w --reps 3 zc: nozc:GCR_ZEROCOPY=0 || exit $?; done
timeout -k 10 300 python -u tools/lat_ab.py --workload f --reps 2 zc: nozc:GCR_ZEROCOPY=0 || exit $?
TAG=${TAG:-r3_s15}b bash tools/r3_s11.sh
