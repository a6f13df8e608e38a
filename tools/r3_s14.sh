#!/bin/bash
set -u
D=gpurun_out/${TAG:-r3_s14}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_summary.py tests/test_gpu_sharded.py tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread > $D/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $D/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lat_ab.py --workload m2 --reps 3 one: three:GCR_SUMMARY_ONE=0 || exit $?
timeout -k 10 300 python -u tools/lat_ab.py --workload h --reps 3 one: three:GCR_SUMMARY_ONE=0 || exit $?
TAG=r3_s14b bash tools/r3_s11.sh
