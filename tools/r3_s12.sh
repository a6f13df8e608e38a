#!/bin/bash
# configs[4] batch: host threads per GPU sweep (default lambda)
set -u
D=gpurun_out/${TAG:-r3_s12}
mkdir -p $D
for c in ${CONC:-8 12 16}; do
  timeout -k 10 400 python bench.py --workload batch --concurrency $c --cpu-seconds 0 --no-hbm-probe > $D/batch_c$c.log 2>&1 || { echo "batch c$c failed"; tail -5 $D/batch_c$c.log; exit 1; }
  tail -n 1 $D/batch_c$c.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('c$c', round(c['problems_per_s'],1), 'problems/s', {k: round(v['ms_total']) for k,v in c['rank0_phase_ms_sums'].items()}, {k: round(v['ms_lo_lists']) for k,v in c['rank0_phase_ms_sums'].items()})"
done
