#!/bin/bash
# Full measurement session on the MI355X box: smoke, GPU tests, the default
# bench line, rocprofv3 kernel stats of the default bench, PMC passes for the
# headline (M2) and the H / F workloads.  Every GPU step has its own limit;
# a crash / abort / timeout ends the session.
set -u
mkdir -p gpurun_out
STEPS="smoke tests bench prof" bash tools/gpu_session.sh || exit $?
for w in m2 h f; do
  PMC_DIR=gpurun_out/pmc_$w BENCH_ARGS="--workload $w --steps 20 --warmup 2 --cpu-seconds 0 --no-latency" \
    bash tools/pmc_session.sh || exit $?
done
for w in h f; do
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$w -o run --output-format csv -- \
    python3 bench.py --workload $w --cpu-seconds 0 --no-latency > gpurun_out/prof_$w.log 2>&1 || exit $?
done
echo "session done"
