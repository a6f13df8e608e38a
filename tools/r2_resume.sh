#!/bin/bash
# Round-2 resume check after a container rebuild: GPU suite and the M2 / H / F
# bench lines at HEAD.  Every GPU step under its own time limit; a crash,
# abort or timeout ends the session.
set -u
O=gpurun_out/resume
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -c 400 "$O/$name.log"; echo
  case $rc in 0|1) return 0 ;; *) echo "fatal rc=$rc"; exit $rc ;; esac
}
step tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
step bench_m2 400 python bench.py --gpus 1 --steps 20 --warmup 5
step bench_h 300 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe
step bench_f 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe
echo "session done"
