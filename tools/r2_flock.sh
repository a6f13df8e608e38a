#!/bin/bash
# F generator with the lockstep cubic root finder and branch-free root
# validation (fund.h): F parity tests, the F bench line and the rocprofv3
# kernel stats of the same bench (k_generate_f's average duration).
set -u
O=gpurun_out/flock
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fundamental.py tests/test_gpu_geo_band.py tests/test_gpu_sharded.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests_f.log 2>&1 || { tail -30 $O/tests_f.log; exit 1; }
tail -3 $O/tests_f.log
timeout -k 10 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe > $O/benchf.log 2>&1 || { tail -20 $O/benchf.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f -o run --output-format csv -- python3 bench.py --workload f --cpu-seconds 0 --no-hbm-probe --no-latency > $O/prof_f.log 2>&1 || { tail -20 $O/prof_f.log; exit 1; }
echo "session done"
