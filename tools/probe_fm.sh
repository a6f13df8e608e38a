#!/bin/bash
# k_score_fm timing probes (GCR_PROBE bits; results invalid when set) and
# A/B builds (LIBS: in-tree libraries, e.g. "libgcr.so libgcr_x.so" from
# `make variant`): the live launch average per setting.
# usage: [PROBES="0 1 ..."] [LIBS="..."] tools/probe_fm.sh [outdir] [workload]
set -u
O=${1:-gpurun_out/probe}; W=${2:-m2}; mkdir -p $O
for lib in ${LIBS:-libgcr.so}; do
for pb in ${PROBES:-0 1 2 3 64 0}; do
  tag=${lib%.so}_$pb
  GCR_LIB=$lib GCR_PROBE=$pb timeout -k 10 120 python -u bench.py --workload $W --steps 400 --warmup 20 --cpu-seconds 0 --no-latency --no-hbm-probe > $O/probe_$tag.log 2>&1 || { tail -5 $O/probe_$tag.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$O/probe_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$lib probe $pb', 'kernel_us %.2f' % (1e3*r['avg_kernel_ms']), 'step_ms %.4f' % d['ms_per_step'])"
done
done
