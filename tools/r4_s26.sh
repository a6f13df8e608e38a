#!/bin/bash
# round-4 session 26: scorer without its VGPR spill -- parity, same-box A/B
# against the previous build (libgcr_base.so), rocprofv3 stats of both
set -u
O=gpurun_out/r4_s26; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_config.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --cpu-seconds 0 --no-latency > $O/b_new$i.log 2>&1 || { tail -5 $O/b_new$i.log; exit 1; }
GCR_LIB=libgcr_base.so timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --cpu-seconds 0 --no-latency > $O/b_base$i.log 2>&1 || { tail -5 $O/b_base$i.log; exit 1; }
done
for f in $O/b_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_kernel_ms"])')"; done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st_new -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-latency > $O/st_new.log 2>&1 || { tail -5 $O/st_new.log; exit 1; }
GCR_LIB=libgcr_base.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st_base -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-latency > $O/st_base.log 2>&1 || { tail -5 $O/st_base.log; exit 1; }
grep -h "k_score_fm<2" $O/st_new/run_kernel_stats.csv $O/st_base/run_kernel_stats.csv | cut -d, -f2-6
