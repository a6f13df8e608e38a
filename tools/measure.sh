#!/bin/bash
# Measurement session (any round): GPU suite, smoke, the driver-shaped bench
# line (M2 with the latency leg and the CPU baseline), the F line, rocprofv3
# kernel stats of both, and the PMC passes of both (tools/pmc_sets_r4.txt, one
# rocprofv3 run per counter set).  Every GPU step has its own time limit; any
# failure ends the session.
#   OUT=gpurun_out/<dir> PART=run|prof|all tools/measure.sh
# PART=run: suite, smoke, bench lines; PART=prof: kernel stats and PMC passes.
set -u
O=${OUT:-gpurun_out/measure}; mkdir -p $O
step() { echo "== $1"; }
PART=${PART:-all}
if [ "$PART" != "prof" ]; then
step suite
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -2 $O/suite.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
step bench_f
timeout -k 10 600 python -u bench.py --workload f --steps 200 --warmup 20 --cpu-seconds 0 > $O/bench_f.log 2>&1 || { tail -20 $O/bench_f.log; exit 1; }
tail -1 $O/bench_f.log > $O/bench_f.json
fi
[ "$PART" = "run" ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step stats_m2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_m2 -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-latency > $O/stats_m2.log 2>&1 || { tail -20 $O/stats_m2.log; exit 1; }
python3 tools/dispatch_span.py $(find $O/stats_m2 -name "*kernel_trace.csv" | head -1) > $O/stats_m2_span.txt && cat $O/stats_m2_span.txt
step stats_m2_one_stream
GCR_VERIFY_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_m2_1s -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-latency > $O/stats_m2_1s.log 2>&1 || { tail -20 $O/stats_m2_1s.log; exit 1; }
python3 tools/dispatch_span.py $(find $O/stats_m2_1s -name "*kernel_trace.csv" | head -1) > $O/stats_m2_1s_span.txt && cat $O/stats_m2_1s_span.txt
step stats_f
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_f -o run --output-format csv -- python3 bench.py --workload f --steps 200 --warmup 20 --cpu-seconds 0 --no-latency > $O/stats_f.log 2>&1 || { tail -20 $O/stats_f.log; exit 1; }
step pmc_m2
PMC_DIR=$O/pmc_m2 PMC_FILE=tools/pmc_sets_r4.txt BENCH_ARGS="--steps 3 --warmup 1 --cpu-seconds 0 --no-latency --no-hbm-probe" tools/pmc_session.sh || exit 1
step pmc_f
PMC_DIR=$O/pmc_f PMC_FILE=tools/pmc_sets_r4.txt BENCH_ARGS="--workload f --steps 3 --warmup 1 --cpu-seconds 0 --no-latency --no-hbm-probe" tools/pmc_session.sh || exit 1
step done
