#!/bin/bash
# round-4 session 15: kernel + memory-copy trace of the M2 latency call
set -u
O=gpurun_out/r4_s15; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/latency_probe.py --reps 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
ls $O/prof
