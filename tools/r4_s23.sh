#!/bin/bash
# round-4 session 23: zero-copy batch records -- verify tests, driver-shaped bench A/B
set -u
O=gpurun_out/r4_s23; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_fundamental.py tests/test_homography.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-latency > $O/b_zc$i.log 2>&1 || { tail -5 $O/b_zc$i.log; exit 1; }
GCR_ZEROCOPY=0 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-latency > $O/b_nozc$i.log 2>&1 || { tail -5 $O/b_nozc$i.log; exit 1; }
done
for f in $O/b_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
