#!/bin/bash
# configs[4] batch under rocprofv3: total kernel time vs wall
set -u
D=gpurun_out/${TAG:-r3_s13}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 python bench.py --workload batch --cpu-seconds 0 --no-hbm-probe > $D/batch.log 2>&1 || { echo "batch failed"; tail -5 $D/batch.log; exit 1; }
tail -n 1 $D/batch.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --workload batch --cpu-seconds 0 --no-hbm-probe > $D/prof.log 2>&1 || { echo "prof failed"; tail -5 $D/prof.log; exit 1; }
f=$(find $D/prof -name "*kernel_stats.csv" | head -1); cp $f $D/kstats.csv
f=$(find $D/prof -name "*kernel_trace.csv" | head -1); cp $f $D/ktrace.csv
echo done
