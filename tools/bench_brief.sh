#!/bin/bash
# one line per bench log: value, ms/step, score-kernel time, latency median
for f in "$@"; do python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], '%.4g'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'kern us %.1f'%(1000*r['avg_kernel_ms']), r['kernel'], 'lat', (d.get('wall_time_to_0.99_confidence') or {}).get('ms_median'))
"; done
