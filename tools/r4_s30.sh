#!/bin/bash
# round-4 session 30: host wait mode A/B (GCR_SCHED, separate processes, interleaved)
set -u
O=gpurun_out/r4_s30; mkdir -p $O
for i in 1 2 3; do
for m in default spin yield; do
GCR_SCHED=$m timeout -k 10 200 python -u tools/lat_ab.py --workload m2 --reps 4 $m: > $O/lat_${m}$i.log 2>&1 || { tail -20 $O/lat_${m}$i.log; exit 1; }
done
done
grep -h "median" $O/lat_*.log | cut -c1-100
