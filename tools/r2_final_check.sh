#!/bin/bash
# Final check of the round-2 HEAD build: GPU suite, smoke(), the driver's
# bench command and the F line with its wall time to 0.99.
set -u
O=gpurun_out/final_check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_m2.log 2>&1 || { tail -20 $O/bench_m2.log; exit 1; }
timeout -k 10 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe > $O/bench_f.log 2>&1 || { tail -20 $O/bench_f.log; exit 1; }
echo "session done"
