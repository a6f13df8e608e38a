#!/bin/bash
# kernel trace of the F and H bench steps
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f -o run -- python3 bench.py --workload f --cpu-seconds 0 --no-hbm-probe --steps 50 --warmup 5 > gpurun_out/proff.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_h -o run -- python3 bench.py --workload h --cpu-seconds 0 --no-hbm-probe --steps 50 --warmup 5 > gpurun_out/profh.log 2>&1
rc=$?
find gpurun_out/prof_f gpurun_out/prof_h -name "*stats*"
exit $rc
