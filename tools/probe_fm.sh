#!/bin/bash
# k_score_fm timing probes (GCR_PROBE bits; results invalid when set): the
# live average launch of the bench workload per probe setting.
# usage: tools/probe_fm.sh [outdir] [workload]; every run has its own limit.
set -u
O=${1:-gpurun_out/probe}; W=${2:-m2}; mkdir -p $O
for pb in ${PROBES:-0 1 2 3 64 0}; do
  GCR_PROBE=$pb timeout -k 10 120 python -u bench.py --workload $W --steps 400 --warmup 20 --cpu-seconds 0 --no-latency --no-hbm-probe > $O/probe_$pb.log 2>&1 || { tail -5 $O/probe_$pb.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$O/probe_$pb.log').read().strip().splitlines()[-1]); r=d['roofline']
print('probe $pb', 'kernel_us %.2f' % (1e3*r['avg_kernel_ms']), 'step_ms %.4f' % d['ms_per_step'])"
done
