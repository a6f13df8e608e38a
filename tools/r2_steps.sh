#!/bin/bash
# ms per step against the number of timed steps (driver uses 20)
set -u
mkdir -p gpurun_out
for k in 20 50 100 200 500 1000 2000; do
  timeout -k 10 120 python bench.py --gpus 1 --steps $k --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > gpurun_out/k_$k.log 2>&1 || exit 1
done
rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_k200 -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > gpurun_out/prof_k200.log 2>&1
echo done
