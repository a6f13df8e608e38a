#!/bin/bash
# Deferred selection, second pass: batches right after a ring flush are no
# longer timed.  Verify tests, the 2000-step M2 line (live kernel time vs
# rocprofv3), and the full default bench line.
set -u
O=gpurun_out/defer2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_config.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 50 --cpu-seconds 0 --no-hbm-probe --no-latency > $O/m2_2000.log 2>&1 || { tail -20 $O/m2_2000.log; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/m2_driver.log 2>&1 || { tail -20 $O/m2_driver.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_m2_2000 -o run --output-format csv -- python3 bench.py --gpus 1 --steps 2000 --warmup 50 --cpu-seconds 0 --no-hbm-probe --no-latency > $O/prof_m2_2000.log 2>&1 || { tail -20 $O/prof_m2_2000.log; exit 1; }
echo "session done"
