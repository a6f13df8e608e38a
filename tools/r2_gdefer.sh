#!/bin/bash
# Deferred selection for the correspondence pipeline (ring of batch buffer
# sets, one selection launch per ring): verify tests, then the H / F lines
# with and without deferral (GCR_VERIFY_DEFER=0), rocprofv3 stats of H.
set -u
O=gpurun_out/gdefer
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_config.py tests/test_homography.py tests/test_fundamental.py tests/test_gpu_sharded.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for d in 1 0; do
  for w in h f; do
    GCR_VERIFY_DEFER=$d timeout -k 10 200 python bench.py --workload $w --cpu-seconds 0 --no-hbm-probe --no-latency > $O/${w}_d$d.log 2>&1 || { tail -20 $O/${w}_d$d.log; exit 1; }
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_h -o run --output-format csv -- python3 bench.py --workload h --cpu-seconds 0 --no-hbm-probe --no-latency > $O/prof_h.log 2>&1 || { tail -20 $O/prof_h.log; exit 1; }
echo "session done"
