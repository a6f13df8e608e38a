#!/bin/bash
# first-chunk size A/B (GCR_FIRST_CHUNK) per seed, M2 / M1 / H, F medians
set -u
D=gpurun_out/r3_fc
mkdir -p $D
for w in m2 m1 h; do timeout -k 10 300 python -u tools/lat_seeds.py --workload $w --reps 3 s256: s128:GCR_FIRST_CHUNK=128 > $D/seeds_$w.log 2>&1 || { echo "$w failed"; tail -5 $D/seeds_$w.log; exit 1; }; echo "== $w"; tail -11 $D/seeds_$w.log | cut -c1-200; done
timeout -k 10 300 python -u tools/lat_ab.py --workload f --reps 2 s256: s128:GCR_FIRST_CHUNK=128 > $D/lat_f.log 2>&1 || exit 1
tail -2 $D/lat_f.log
