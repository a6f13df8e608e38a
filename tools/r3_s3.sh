#!/bin/bash
# Full GPU suite + smoke + the bench lines (driver's M2 command, F, H, strong N=1).
set -u
D=gpurun_out/${TAG:-r3_s3}
mkdir -p $D
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$D/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n ${TAILN:-4} "$D/$name.log"
    case $rc in 0|1|5) return 0 ;; *) echo "fatal rc=$rc, stopping"; exit $rc ;; esac
}
[ -n "${NOTESTS:-}" ] || run tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
[ -n "${NOTESTS:-}" ] || run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_m2 400 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_f 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe
run bench_h 300 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe
run strong1 300 python bench.py --mode strong --steps 16 --warmup 2
echo "session done"
