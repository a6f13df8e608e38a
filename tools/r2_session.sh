#!/bin/bash
# Round-2 GPU session: GPU tests, the driver's bench line, the launcher's
# 2-rank rehearsal (gloo, ranks share device 0) and the strong-scaling mode.
set -u
mkdir -p gpurun_out
STEPS="${STEPS:-tests bench}" BENCH_ARGS="${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5}" \
  PYTEST_ARGS="${PYTEST_ARGS:---timeout 300}" bash tools/gpu_session.sh || exit $?
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -c 2500 "gpurun_out/$name.log"; echo
  [ $rc -eq 0 ] || exit $rc
}
[ -n "${NO_EXTRA:-}" ] && exit 0
step bench_g2 300 python bench.py --gpus 2 --steps 20 --warmup 5 --cpu-seconds 0 --no-latency
step strong1 300 python bench.py --mode strong --steps 8 --warmup 1
step strong2 300 python bench.py --mode strong --gpus 2 --steps 8 --warmup 1
echo "session done"
