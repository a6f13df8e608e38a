set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python tools/latency_probe.py --reps 10 > gpurun_out/latency.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/latency.log; exit 1; }
tail -1 gpurun_out/latency.log
