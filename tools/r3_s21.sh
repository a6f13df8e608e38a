#!/bin/bash
# DPP summary scans + speculative-chunk trim: summary / sharded / full GPU
# suite, latency A/B (trim on / off), kernel trace of the M2 latency call.
set -u
D=gpurun_out/r3_s21
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_summary.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread > $D/sum_tests.log 2>&1; rc=$?
echo "summary tests rc=$rc"; tail -2 $D/sum_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $D/tests.log
[ $rc -eq 0 ] || exit $rc
for w in m2 m1 h; do timeout -k 10 300 python -u tools/lat_ab.py --workload $w --reps 4 trim: notrim:GCR_SPEC_TRIM=0 > $D/lat_$w.log 2>&1 || { echo "lat $w failed"; tail -5 $D/lat_$w.log; exit 1; }; tail -2 $D/lat_$w.log; done
timeout -k 10 300 python -u tools/lat_ab.py --workload f --reps 2 trim: notrim:GCR_SPEC_TRIM=0 > $D/lat_f.log 2>&1 || { echo "lat f failed"; exit 1; }
tail -2 $D/lat_f.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python3 tools/latency_probe.py --reps 6 > $D/trace.log 2>&1 || { echo "trace failed"; exit 1; }
tail -1 $D/trace.log
