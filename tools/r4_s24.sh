#!/bin/bash
# round-4 session 24: kernel + copy trace of the driver-shaped 20-step bench call
set -u
O=gpurun_out/r4_s24; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log | cut -c1-200
