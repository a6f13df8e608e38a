#!/bin/bash
# round-4 session 16: fold walk stamps; driver-shaped bench line (M2, latency leg)
set -u
O=gpurun_out/r4_s16; mkdir -p $O
timeout -k 10 120 python -u tools/fold_bench.py > $O/fold_bench.log 2>&1 || { cat $O/fold_bench.log; exit 1; }
cat $O/fold_bench.log
timeout -k 10 400 python -u bench.py --steps 50 --warmup 10 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step')}, d.get('latency', d.get('config')))"
