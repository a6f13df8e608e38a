#!/bin/bash
# Round-2 full session: all GPU tests, the driver's bench line (+ latency leg),
# strong-mode lines with and without the speculative prefetch, the latency
# kernel/copy trace.
set -u
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -c 1500 "gpurun_out/$name.log"; echo
  case $rc in 0|1) return 0 ;; *) echo "fatal rc=$rc"; exit $rc ;; esac
}
step tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
step strong1 300 python bench.py --mode strong --steps 16 --warmup 4
step strong1_nopf 300 env GCR_PREFETCH=0 python bench.py --mode strong --steps 16 --warmup 4
step benchf 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe
step benchf_nopf 300 env GCR_PREFETCH=0 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe
echo "session done"
