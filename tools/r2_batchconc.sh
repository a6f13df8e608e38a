#!/bin/bash
# configs[4] batch: host threads per GPU (--concurrency 4 / 8 / 12 / 16);
# F wall time to 0.99 with the generator's lanes per slot forced (GCR_GEN_G
# = 2 / 4 / 8 / 16, widening groups) -- the replay path's large chunks use 2.
set -u
O=gpurun_out/bconc
mkdir -p $O
for c in 4 8 12 16; do
  timeout -k 10 300 python bench.py --workload batch --concurrency $c --cpu-seconds 0 --no-hbm-probe > $O/batch_c$c.log 2>&1 || { tail -20 $O/batch_c$c.log; exit 1; }
done
for g in 2 4 8 16; do
  GCR_GEN_G=$g timeout -k 10 300 python bench.py --workload f --steps 20 --warmup 5 --cpu-seconds 0 --no-hbm-probe > $O/flat_g$g.log 2>&1 || { tail -20 $O/flat_g$g.log; exit 1; }
done
echo "session done"
