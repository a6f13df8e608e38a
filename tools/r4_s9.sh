set -u
O=gpurun_out/r4_s9; mkdir -p $O
run() { local n=$1 to=$2; shift 2; echo "=== $n"; timeout -k 10 $to "$@" > $O/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -n 6 $O/$n.log; case $rc in 0|1) ;; *) exit $rc;; esac; }
run tests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
run lat 300 python -u tools/lat_ab.py --workload m2 --reps 4 base: seq:GCR_LO_FOLD=seq
export TMPDIR=/tmp
run proflat 300 rocprofv3 --kernel-trace --stats -d $O/prof_lat -o run --output-format csv -- python3 tools/latency_probe.py --reps 5
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open("gpurun_out/r4_s9/prof_lat/run_kernel_stats.csv")))
for r in rows[:12]: print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"])/1000,2), "us")
PY
