#!/bin/bash
# Refit / latency session: the refit parity tests, the bench's latency leg
# (M2, 11 calls to 0.99 confidence) and a rocprofv3 kernel + copy trace of it.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -k "refit" --timeout 300 > gpurun_out/refit_tests.log 2>&1
rc=$?; tail -5 gpurun_out/refit_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-hbm-probe > gpurun_out/lat_bench.log 2>&1 || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/lat_bench.log').read().strip().splitlines()[-1]);print(json.dumps(d['wall_time_to_0.99_confidence']))"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_lat -o run --output-format csv -- python3 tools/latency_probe.py --reps 5 > gpurun_out/prof_lat.log 2>&1 || exit $?
echo "session done"
