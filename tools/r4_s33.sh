#!/bin/bash
# round-4 session 33: rocprofv3 --kernel-trace --stats of the driver's exact bench command
set -u
O=gpurun_out/r4_s33; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -v "^[EW]2026" $O/bench.log | tail -1 > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'])"
grep -h "k_score_fm<2" $O/prof/run_kernel_stats.csv | cut -d, -f2-4
