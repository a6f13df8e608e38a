#!/bin/bash
# Round-5 GPU session.  STEPS selects the parts (default: suite lat bench).
#   suite  GPU test suite (TESTS: pytest selection, default tests -m gpu)
#   smoke  __graft_entry__.smoke()
#   lat    tools/lat_seeds.py per-seed latency (LAT_SETS: its settings)
#   bench  python bench.py (BENCH_ARGS)
#   benchf bench.py --workload f
#   stats  rocprofv3 --kernel-trace --stats of bench.py (BENCH_ARGS) into $O/stats
#   trace  tools/lo_trace.py host timeline of the LO rounds
#   latst  rocprofv3 --kernel-trace --stats of the latency leg only
# Every GPU step has its own time limit; any failure ends the session.
set -u
O=${OUT:-gpurun_out/r5}; mkdir -p $O
STEPS=${STEPS:-"suite lat bench"}
fail() { echo "!! $1 rc=$2"; tail -40 "$3"; exit 1; }
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
    suite) timeout -k 10 ${SUITE_TO:-900} python -u -m pytest ${TESTS:-tests -m gpu} -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || fail suite $? $O/suite.log; tail -2 $O/suite.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $? $O/smoke.log; tail -1 $O/smoke.log ;;
    lat) timeout -k 10 400 python -u tools/lat_seeds.py --workload ${LAT_WL:-m2} --reps ${LAT_REPS:-3} ${LAT_SETS:-base:} > $O/lat_${LAT_WL:-m2}.log 2>&1 || fail lat $? $O/lat_${LAT_WL:-m2}.log; cat $O/lat_${LAT_WL:-m2}.log ;;
    bench) timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || fail bench $? $O/bench.log; tail -1 $O/bench.log > $O/bench.json; python3 -c "import json;d=json.load(open('$O/bench.json'));w=d.get('wall_time_to_0.99_confidence',{});print(d['value'],d['ms_per_step'],d['roofline'].get('frac'),d['roofline'].get('avg_kernel_ms'),w.get('ms_median'),max(w.get('ms_all',[0])))" ;;
    benchf) timeout -k 10 600 python -u bench.py --workload f --steps 200 --warmup 20 --cpu-seconds 0 > $O/bench_f.log 2>&1 || fail benchf $? $O/bench_f.log; tail -1 $O/bench_f.log > $O/bench_f.json; python3 -c "import json;d=json.load(open('$O/bench_f.json'));w=d.get('wall_time_to_0.99_confidence',{});print(d['value'],d['ms_per_step'],w.get('ms_median'),max(w.get('ms_all',[0])))" ;;
    stats) (cd /tmp && true); export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --cpu-seconds 0 ${BENCH_ARGS:-} > $O/stats.log 2>&1 || fail stats $? $O/stats.log; find $O/stats -name '*kernel_stats.csv' -exec head -20 {} \; ;;
    sync) timeout -k 10 120 tools/micro/sync_latency.bin > $O/sync.log 2>&1 || fail sync $? $O/sync.log; cat $O/sync.log ;;
    valu) timeout -k 10 200 tools/micro/valu_issue.bin > $O/valu.log 2>&1 || fail valu $? $O/valu.log; cat $O/valu.log ;;
    trace) GCR_LO_TRACE=1 timeout -k 10 200 python -u tools/lo_trace.py ${LAT_WL:-m2} 2> $O/trace.txt > $O/trace.log || fail trace $? $O/trace.log; python3 tools/lo_trace.py --parse $O/trace.txt ;;
    latst) export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/latst -o run --output-format csv -- python3 tools/lat_seeds.py --workload ${LAT_WL:-m2} --reps 2 base: > $O/latst.log 2>&1 || fail latst $? $O/latst.log; find $O/latst -name '*kernel_stats.csv' -exec head -25 {} \; ;;
  esac
done
echo "== done $(date +%T)"
