set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_lat -o run --output-format csv -- python3 tools/latency_probe.py --reps 5 > gpurun_out/prof_lat.log 2>&1
