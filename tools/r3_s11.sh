#!/bin/bash
# configs[4] batch: default lambda and 0, with the context pool / pair cells
set -u
D=gpurun_out/${TAG:-r3_s11}
mkdir -p $D
for l in def 0; do
  a=""; [ $l = 0 ] && a="--batch-lambda 0"
  timeout -k 10 400 python bench.py --workload batch $a --cpu-seconds 0 --no-hbm-probe > $D/batch_$l.log 2>&1 || { echo "batch $l failed"; tail -5 $D/batch_$l.log; exit 1; }
  tail -n 1 $D/batch_$l.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('$l', round(c['problems_per_s'],1), 'problems/s', {k: round(v['ms_total']) for k,v in c['rank0_phase_ms_sums'].items()}, {k: round(v['ms_lo_lists']) for k,v in c['rank0_phase_ms_sums'].items()})"
done
