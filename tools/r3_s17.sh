#!/bin/bash
set -u
D=gpurun_out/${TAG:-r3_s17}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_summary.py tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $D/tests.log
[ $rc -eq 0 ] || exit $rc
for w in m2 h; do timeout -k 10 300 python -u tools/lat_ab.py --workload $w --reps 3 spin: block:GCR_SYNC=block || exit $?; done
timeout -k 10 300 python -u tools/lat_ab.py --workload f --reps 2 spin: block:GCR_SYNC=block || exit $?
TAG=${TAG:-r3_s17}b bash tools/r3_s11.sh
