#!/bin/bash
# round-4 session 21: zero-copy A/B of the split small scorer (kernel trace of both)
set -u
O=gpurun_out/r4_s21; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/zc -o run --output-format csv -- python3 tools/latency_probe.py --reps 5 > $O/zc.log 2>&1 || { tail -20 $O/zc.log; exit 1; }
GCR_ZEROCOPY=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/nozc -o run --output-format csv -- python3 tools/latency_probe.py --reps 5 > $O/nozc.log 2>&1 || { tail -20 $O/nozc.log; exit 1; }
for d in zc nozc; do echo "== $d"; grep -h "k_lo_fold<2>\|k_lo_resid<2>\|sift_gram" $O/$d/run_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-40,150-; done
timeout -k 10 300 python -u tools/lat_ab.py --workload m2 --reps 5 base: nozc:GCR_ZEROCOPY=0 > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
cat $O/lat.log
