#!/bin/bash
# round-4 session 27: look-ahead generator lanes per slot (GCR_GEN_LANES) sweep, 200-step M2 bench
set -u
O=gpurun_out/r4_s27; mkdir -p $O
for i in 1 2; do
for g in 16 8 32 64; do
GCR_GEN_LANES=$g timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --cpu-seconds 0 --no-latency > $O/b_g${g}_$i.log 2>&1 || { tail -5 $O/b_g${g}_$i.log; exit 1; }
done
done
for f in $O/b_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_kernel_ms"])')"; done
