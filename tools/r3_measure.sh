#!/bin/bash
# Round-3 measurement session for one workload: GCR_PROBE timing breakdown
# (results invalid under a probe; only times are read), the rocprofv3 --stats
# summary of a bench run, and the PMC passes (FETCH / WRITE / SQ) that
# profiles/pmc_traffic.json is built from.  Each GPU step has its own limit;
# any failure ends the session.
#   WL=m2|m1|h|f  SLOTS=4096  TAG=r3_x  PROBES="0 1 2 4 8"
set -u
WL="${WL:-m2}"; TAG="${TAG:-r3}"; SLOTS="${SLOTS:-}"
D=gpurun_out/$TAG
mkdir -p "$D"
SA=""; [ -n "$SLOTS" ] && SA="--slots $SLOTS"
for p in ${PROBES:-0}; do
  GCR_PROBE=$p timeout -k 10 180 python bench.py --workload $WL $SA --steps 2000 --warmup 20 --cpu-seconds 0 --no-latency --no-hbm-probe > "$D/probe_$p.json" 2> "$D/probe_$p.err" || { echo "probe $p rc=$?"; tail -5 "$D/probe_$p.err"; exit 1; }
  python - "$D/probe_$p.json" "$p" <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"probe {sys.argv[2]}: step {d['ms_per_step']*1e3:.1f} us, kernel {d['roofline']['avg_kernel_ms']*1e3:.1f} us, {d['value']:.4g} hyp/s")
P
done
if [ -n "${STATS:-1}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$D/prof" -o run --output-format csv -- python3 bench.py --workload $WL $SA --steps 2000 --warmup 20 --cpu-seconds 0 --no-latency --no-hbm-probe > "$D/prof.log" 2>&1 || { echo "prof rc=$?"; tail -5 "$D/prof.log"; exit 1; }
  find "$D/prof" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$D/kernel_stats.csv"
  head -4 "$D/kernel_stats.csv"
fi
if [ -n "${PMC:-1}" ]; then
  PMC_DIR="$D/pmc" PMC_FILE=tools/pmc_sets_r3.txt BENCH_ARGS="--workload $WL $SA --steps 200 --warmup 20 --cpu-seconds 0 --no-latency --no-hbm-probe" bash tools/pmc_session.sh > "$D/pmc.log" 2>&1 || { echo "pmc failed"; tail -20 "$D/pmc.log"; exit 1; }
  echo "pmc ok"
fi
echo "session $TAG done"
