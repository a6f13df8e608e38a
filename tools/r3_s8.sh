#!/bin/bash
# kernel times of the small-batch scorer (k_lo_fold vs k_lo_chain) in the M2 latency call
set -u
D=gpurun_out/${TAG:-r3_s8}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for s in ${SETS:-fold seq}; do
  env_=""; [ $s = seq ] && env_="GCR_LO_FOLD=seq"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$s -o run --output-format csv -- python3 tools/lat_ab.py --workload ${WL:-m2} --reps 1 "$s:$env_" > $D/prof_$s.log 2>&1 || { echo "prof $s failed"; tail -5 $D/prof_$s.log; exit 1; }
  f=$(find $D/prof_$s -name "*kernel_stats.csv" | head -1); cp $f $D/kstats_$s.csv
  echo "== $s"; cut -d, -f1-4 $D/kstats_$s.csv | head -12 | cut -c1-200
done
