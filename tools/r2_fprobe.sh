#!/bin/bash
# correspondence scorers: chain cost (GCR_PROBE=1 skips the fold; results invalid)
set -u
mkdir -p gpurun_out
for w in f h; do
for p in 0 1 2 4; do
  GCR_VERIFY_PIPE=0 GCR_PROBE=$p timeout -k 10 300 python bench.py --workload $w --cpu-seconds 0 --no-hbm-probe --no-latency > gpurun_out/fp_${w}_$p.log 2>&1 || exit 1
done
done
echo done
