#!/bin/bash
# driver-shaped bench line (--steps 20 --warmup 5) under timing strides
set -u
mkdir -p gpurun_out
for rep in 1 2 3; do
for st in 1 4 20; do
  GCR_TIMING_STRIDE=$st timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > gpurun_out/st_${st}_$rep.log 2>&1 || exit 1
done
done
for st in 1 32; do
  GCR_TIMING_STRIDE=$st timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 5 --cpu-seconds 0 --no-latency --no-hbm-probe > gpurun_out/st200_${st}.log 2>&1 || exit 1
done
echo done
