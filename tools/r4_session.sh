#!/bin/bash
# Round-4 GPU session: VALU issue micro-benchmark, the GPU suite, latency A/B
# (split segment fold vs one-lane fold) on M2 and F, the bench, a rocprofv3
# kernel-trace summary.  Each GPU step has its own time limit; a crash / abort
# / timeout stops the session, an ordinary test failure does not.
set -u
OUT=${OUT:-gpurun_out/r4}
mkdir -p "$OUT"
STEPS="${STEPS:-micro tests latm2 latf bench prof}"
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 12 "$OUT/$name.log"
    case $rc in 0|1|5) return 0 ;; *) echo "fatal rc=$rc, stopping"; exit $rc ;; esac
}
for s in $STEPS; do
  case $s in
    micro) run micro 120 ./tools/micro/valu_issue.bin ;;
    smoke) run smoke 300 python __graft_entry__.py ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ;;
    latm2) run latm2 300 python -u tools/lat_ab.py --workload m2 --reps 5 base: seq:GCR_LO_FOLD=seq ;;
    latf)  run latf 300 python -u tools/lat_ab.py --workload f --reps 3 base: seq:GCR_LO_FOLD=seq ;;
    bench) run bench 600 python -u bench.py ${BENCH_ARGS:-} ;;
    prof)  export TMPDIR=/tmp
           run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --no-latency ${BENCH_ARGS:-} ;;
  esac
done
