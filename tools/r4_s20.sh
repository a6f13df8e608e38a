#!/bin/bash
# round-4 session 20: Gram refit pair-row shortcut -- refit parity tests, frozen pins, latency trace
set -u
O=gpurun_out/r4_s20; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_frozen_pin.py -x -q -k "refit or gram or frozen" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/latency_probe.py --reps 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -h "sift_gram\|k_lo_fold<2>\|k_lo_resid<2>" $O/prof/run_kernel_stats.csv | cut -c1-60,200-330
timeout -k 10 300 python -u tools/lat_ab.py --workload m2 --reps 5 base: > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
cat $O/lat.log
