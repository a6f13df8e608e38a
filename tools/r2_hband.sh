#!/bin/bash
# Homography packed-fp32 pre-band: full GPU suite, then the H bench line with
# the pre-band and with the fp64 band (GCR_PROBE=128), rocprofv3 kernel stats
# of the H line, and the F line at the new default generator (with latency).
set -u
O=gpurun_out/hband
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe > $O/bench_h.log 2>&1 || { tail -20 $O/bench_h.log; exit 1; }
GCR_PROBE=128 timeout -k 10 200 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe --no-latency > $O/bench_h_fp64.log 2>&1 || { tail -20 $O/bench_h_fp64.log; exit 1; }
timeout -k 10 200 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe > $O/bench_f.log 2>&1 || { tail -20 $O/bench_f.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_h -o run --output-format csv -- python3 bench.py --workload h --cpu-seconds 0 --no-hbm-probe --no-latency > $O/prof_h.log 2>&1 || { tail -20 $O/prof_h.log; exit 1; }
GCR_PROBE=128 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_h_fp64 -o run --output-format csv -- python3 bench.py --workload h --cpu-seconds 0 --no-hbm-probe --no-latency > $O/prof_h_fp64.log 2>&1 || { tail -20 $O/prof_h_fp64.log; exit 1; }
echo "session done"
