#!/bin/bash
# round-4 session 25: span timing of the fused launches -- driver-shaped bench A/B
set -u
O=gpurun_out/r4_s25; mkdir -p $O
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-latency > $O/b_span$i.log 2>&1 || { tail -5 $O/b_span$i.log; exit 1; }
GCR_TIMING_SPAN=0 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-latency > $O/b_pairs$i.log 2>&1 || { tail -5 $O/b_pairs$i.log; exit 1; }
done
for f in $O/b_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_kernel_ms"], d["roofline"]["frac"])')"; done
