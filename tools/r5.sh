#!/bin/bash
# Round-5 GPU session.  STEPS selects the parts (default: suite lat bench).
#   suite  GPU test suite (TESTS: pytest selection, default tests -m gpu)
#   smoke  __graft_entry__.smoke()
#   lat    tools/lat_seeds.py per-seed latency (LAT_SETS: its settings)
#   bench  python bench.py (BENCH_ARGS)
#   benchf bench.py --workload f
#   stats  rocprofv3 --kernel-trace --stats of bench.py (BENCH_ARGS) into $O/stats
#   trace  tools/lo_trace.py host timeline of the LO rounds (per TRACE_ENVS entry)
#   ktrace rocprofv3 kernel trace of the latency leg, one call's dispatch timeline
#   pmclat rocprofv3 --pmc passes (PMC_FILE lines) over the latency leg, kernels matching PMC_MATCH
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
    trace) for te in ${TRACE_ENVS:-X=0}; do echo "-- $te"; env $te GCR_LO_TRACE=1 timeout -k 10 200 python -u tools/lo_trace.py ${LAT_WL:-m2} 2> $O/trace_$te.txt > $O/trace.log || fail trace $? $O/trace.log; python3 tools/lo_trace.py --parse $O/trace_$te.txt; done ;;
    ktrace) export TMPDIR=/tmp; for te in ${KTRACE_ENVS:-X=0}; do echo "-- $te"; export $te; timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ktrace_$te -o run --output-format csv -- python3 tools/lat_seeds.py --workload ${LAT_WL:-m2} --reps 1 base: > $O/ktrace.log 2>&1 || fail ktrace $? $O/ktrace.log; python3 tools/trace_gaps.py $(find $O/ktrace_$te -name '*kernel_trace.csv' | head -1) --summary; done ;;
    pmclat) export TMPDIR=/tmp; i=0; while IFS= read -r ctrs; do [ -z "$ctrs" ] && continue; i=$((i+1)); echo "-- pass$i: $ctrs"; timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $O/pmclat$i -o run -- python3 tools/lat_seeds.py --workload ${LAT_WL:-m2} --reps 1 base: > $O/pmclat$i.log 2>&1 || fail pmclat $? $O/pmclat$i.log; python3 tools/pmc_kernel.py $(find $O/pmclat$i -name '*counter_collection.csv' | head -1) --match "${PMC_MATCH:-.}"; done < ${PMC_FILE:-tools/pmc_lat.txt} ;;
    latst) export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/latst -o run --output-format csv -- python3 tools/lat_seeds.py --workload ${LAT_WL:-m2} --reps 2 base: > $O/latst.log 2>&1 || fail latst $? $O/latst.log; find $O/latst -name '*kernel_stats.csv' -exec head -25 {} \; ;;
  esac
done
echo "== done $(date +%T)"
