#!/bin/bash
# Deferred batch selection (one k_select_wg launch per ring of fused batches):
# verify parity tests, then the driver-shaped M2 line (20 steps) and a
# 2000-step line with and without deferral (GCR_VERIFY_DEFER=0), and the
# rocprofv3 kernel stats of the driver-shaped line.
set -u
O=gpurun_out/defer
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for d in 1 0; do
  GCR_VERIFY_DEFER=$d timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-hbm-probe --no-latency > $O/m2_20_d$d.log 2>&1 || { tail -20 $O/m2_20_d$d.log; exit 1; }
  GCR_VERIFY_DEFER=$d timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 50 --cpu-seconds 0 --no-hbm-probe --no-latency > $O/m2_2000_d$d.log 2>&1 || { tail -20 $O/m2_2000_d$d.log; exit 1; }
  GCR_VERIFY_DEFER=$d timeout -k 10 200 python bench.py --workload m1 --cpu-seconds 0 --no-hbm-probe --no-latency > $O/m1_d$d.log 2>&1 || { tail -20 $O/m1_d$d.log; exit 1; }
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_m2 -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-hbm-probe > $O/prof_m2.log 2>&1 || { tail -20 $O/prof_m2.log; exit 1; }
echo "session done"
