#!/bin/bash
# round-4 session 32: the other BASELINE configs on the final kernels -- M1, H, configs[4] batch, strong mode
set -u
O=gpurun_out/r4_s32; mkdir -p $O
timeout -k 10 400 python -u bench.py --workload m1 --steps 200 --warmup 20 --cpu-seconds 0 > $O/m1.log 2>&1 || { tail -5 $O/m1.log; exit 1; }
timeout -k 10 400 python -u bench.py --workload h --steps 200 --warmup 20 --cpu-seconds 0 > $O/h.log 2>&1 || { tail -5 $O/h.log; exit 1; }
timeout -k 10 600 python -u bench.py --workload batch --cpu-seconds 0 > $O/batch.log 2>&1 || { tail -5 $O/batch.log; exit 1; }
timeout -k 10 400 python -u bench.py --mode strong --steps 20 --warmup 5 --cpu-seconds 0 --no-latency > $O/strong.log 2>&1 || { tail -5 $O/strong.log; exit 1; }
for f in m1 h batch strong; do tail -1 $O/$f.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); w=d.get('wall_time_to_0.99_confidence') or {}
print('$f', d['metric'], '%.4g'%d['value'], d['unit'], 'ms/step %.4f'%d['ms_per_step'], 'lat %s'%(round(w['ms_median'],3) if w.get('ms_median') else None))"; done
