#!/bin/bash
# One GPU session on the MI355X box: smoke, parity tests, bench, rocprofv3.
# Each GPU step has its own time limit; a crash/abort/timeout stops the session,
# an ordinary test failure does not.
set -u
mkdir -p gpurun_out
STEPS="${STEPS:-smoke tests bench prof}"
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    case $rc in 0|1|5) return 0 ;; *) echo "fatal rc=$rc, stopping"; exit $rc ;; esac
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python __graft_entry__.py ;;
    tests) run tests ${TESTS_TO:-1200} python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} ;;
    bench) run bench 600 python bench.py ${BENCH_ARGS:-} ;;
    sweep) i=0; while IFS= read -r line; do [ -z "$line" ] && continue; i=$((i+1));
             run "sweep$i" 300 env $line ; done < "${SWEEP_FILE:-tools/sweep.txt}" ;;
    prof)  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
           run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --no-latency ${BENCH_ARGS:-} ;;
  esac
done
