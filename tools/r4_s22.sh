#!/bin/bash
# round-4 session 22: kernel-argument models of the split small scorer (kernel trace of both)
set -u
O=gpurun_out/r4_s22; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_parity.py tests/test_gpu_refit_reuse.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/zc -o run --output-format csv -- python3 tools/latency_probe.py --reps 5 > $O/zc.log 2>&1 || { tail -20 $O/zc.log; exit 1; }
GCR_LO_ARGMODELS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/nozc -o run --output-format csv -- python3 tools/latency_probe.py --reps 5 > $O/nozc.log 2>&1 || { tail -20 $O/nozc.log; exit 1; }
for d in zc nozc; do echo "== $d"; grep -h "k_lo_fold<2>\|k_lo_resid<2>\|sift_gram" $O/$d/run_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-40,150-; done
timeout -k 10 300 python -u tools/lat_ab.py --workload m2 --reps 5 base: noarg:GCR_LO_ARGMODELS=0 > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
cat $O/lat.log
