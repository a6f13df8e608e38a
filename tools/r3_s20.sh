#!/bin/bash
# Kernel + copy trace of the M2 latency call (wide vs one-lane LO fold)
set -u
D=gpurun_out/r3_s20
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for m in wide seq; do
  e=""; [ $m = wide ] && e=wide
  GCR_LO_FOLD=$e timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $D/$m -o run --output-format csv -- python3 tools/latency_probe.py --reps 6 > $D/$m.log 2>&1 || { echo "$m failed"; tail -5 $D/$m.log; exit 1; }
  tail -1 $D/$m.log
done
