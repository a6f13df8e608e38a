#!/bin/bash
# GPU suite, F latency A/B (speculative chunks / chunk cap), configs[4] batch
# with phase sums at the default lambda and at 0, and with pool spinning off.
set -u
D=gpurun_out/${TAG:-r3_s10}
mkdir -p $D
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$D/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n ${TAILN:-2} "$D/$name.log" | cut -c1-400
    case $rc in 0|1|5) return 0 ;; *) echo "fatal rc=$rc, stopping"; exit $rc ;; esac
}
[ -n "${NOTESTS:-}" ] || run tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
run ab_f 400 python -u tools/lat_ab.py --workload f --reps 2 --json $D/ab_f.json all: nospec:GCR_SPECULATE=0 nocap:GCR_CHUNK_CAP=0 neither:GCR_SPECULATE=0,GCR_CHUNK_CAP=0
run ab_h 300 python -u tools/lat_ab.py --workload h --reps 2 --json $D/ab_h.json all: neither:GCR_SPECULATE=0,GCR_CHUNK_CAP=0
run batch 400 python bench.py --workload batch --cpu-seconds 0 --no-hbm-probe
run batch_l0 400 python bench.py --workload batch --batch-lambda 0 --cpu-seconds 0 --no-hbm-probe
echo "session done"
