#!/bin/bash
# configs[4] batch: host pool size (GCR_HOST_THREADS) x problems in flight
# (--concurrency); the driver's smoke() first.
set -u
O=gpurun_out/bpool
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for cfg in 1:8 1:16 4:8 8:8 16:8 4:12; do
  t=${cfg%%:*}; c=${cfg##*:}
  GCR_HOST_THREADS=$t timeout -k 10 300 python bench.py --workload batch --concurrency $c --cpu-seconds 0 --no-hbm-probe > $O/b_t${t}_c$c.log 2>&1 || { tail -20 $O/b_t${t}_c$c.log; exit 1; }
done
echo "session done"
