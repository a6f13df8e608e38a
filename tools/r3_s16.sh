#!/bin/bash
# kernel timeline of M2 latency calls (rocprofv3 kernel + memory-copy trace)
set -u
D=gpurun_out/${TAG:-r3_s16}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $D/tests.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $D/prof -o run --output-format csv -- python3 tools/lat_ab.py --workload ${WL:-m2} --reps 1 base: > $D/prof.log 2>&1 || { echo "prof failed"; tail -5 $D/prof.log; exit 1; }
for f in kernel_trace memory_copy_trace; do g=$(find $D/prof -name "*${f}.csv" | head -1); [ -n "$g" ] && cp $g $D/$f.csv; done
tail -2 $D/prof.log
