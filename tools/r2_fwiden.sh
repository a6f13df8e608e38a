#!/bin/bash
# F generator A/B: widening groups (k_generate_fw) at G = 8 / 16 / 32 against
# fixed groups (GCR_GEN_WIDEN=0), G = 4 / 64, and the previous commit's library
# (libgcr_head.so).  F parity tests first; per variant the F bench line and
# the rocprofv3 kernel stats of the same bench.
set -u
O=gpurun_out/fwiden
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fundamental.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests_f.log 2>&1 || { tail -30 $O/tests_f.log; exit 1; }
tail -3 $O/tests_f.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name env...
  local name=$1; shift
  local lat=--no-latency
  case $name in head|w32) lat= ;; esac
  env "$@" timeout -k 10 200 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe $lat > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; exit 1; }
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$name -o run --output-format csv -- python3 bench.py --workload f --cpu-seconds 0 --no-hbm-probe --no-latency > $O/prof_$name.log 2>&1 || { tail -20 $O/prof_$name.log; exit 1; }
  echo "$name done"
}
run head GCR_LIB=libgcr_head.so
run fixed32 GCR_GEN_WIDEN=0
run w32 GCR_GEN_G=32
run w16 GCR_GEN_G=16
run w8 GCR_GEN_G=8
run w64 GCR_GEN_G=64
run w4 GCR_GEN_G=4
echo "session done"
