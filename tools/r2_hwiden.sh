#!/bin/bash
# Homography generator A/B: widening groups (GCR_GEN_HWIDEN=1) at G = 4 / 8 /
# 16 against the fixed-group k_generate<3, 16>.  Generator parity tests
# first; per variant the H bench line and rocprofv3 kernel stats.
set -u
O=gpurun_out/hwiden
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_homography.py tests/test_fundamental.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe --no-latency > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; exit 1; }
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$name -o run --output-format csv -- python3 bench.py --workload h --cpu-seconds 0 --no-hbm-probe --no-latency > $O/prof_$name.log 2>&1 || { tail -20 $O/prof_$name.log; exit 1; }
  echo "$name done"
}
run fixed16 GCR_GEN_HWIDEN=0
run w16 GCR_GEN_HWIDEN=1 GCR_GEN_G=16
run w8 GCR_GEN_HWIDEN=1 GCR_GEN_G=8
run w4 GCR_GEN_HWIDEN=1 GCR_GEN_G=4
run w2 GCR_GEN_HWIDEN=1 GCR_GEN_G=2
echo "session done"
