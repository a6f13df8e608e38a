#!/bin/bash
# LO fold kernel tests + latency A/B (one process per workload, settings interleaved)
set -u
D=gpurun_out/${TAG:-r3_s6}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_lo_fold.py tests/test_gpu_parity.py tests/test_gpu_summary.py -q -x --timeout 120 --timeout-method thread > $D/tests.log 2>&1; rc=$?
tail -3 $D/tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
timeout -k 10 300 python -u tools/lat_ab.py --workload m2 --reps 3 --json $D/ab_m2.json fold: seq:GCR_LO_FOLD=seq || exit $?
timeout -k 10 300 python -u tools/lat_ab.py --workload h --reps 3 --json $D/ab_h.json fold: seq:GCR_LO_FOLD=seq || exit $?
timeout -k 10 400 python -u tools/lat_ab.py --workload f --reps 2 --json $D/ab_f.json all: nospec:GCR_SPECULATE=0 nocap:GCR_CHUNK_CAP=0 neither:GCR_SPECULATE=0,GCR_CHUNK_CAP=0 seq:GCR_LO_FOLD=seq || exit $?
echo "session done"
