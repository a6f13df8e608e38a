#!/bin/bash
# Summary replay session: its A/B test against the per-slot replay, the
# parity suites that run the default (summary) path, the sharded tests, and
# skeleton probes of k_score_fm.  A test failure does not stop the session; a
# crash, abort or time limit does.
set -u
D=gpurun_out/${TAG:-r3_s2}
mkdir -p $D
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$D/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 15 "$D/$name.log"
    case $rc in 0|1|5) return 0 ;; *) echo "fatal rc=$rc, stopping"; exit $rc ;; esac
}
PT="python -u -m pytest -q -rf --timeout 300 --timeout-method thread"
run summary 900 $PT tests/test_gpu_summary.py -x
run parity 900 $PT -m gpu tests/test_golden.py tests/test_golden_corr.py tests/test_frozen_pin.py tests/test_fundamental.py tests/test_homography.py tests/test_gpu_parity.py tests/test_gpu_graphcut.py
run sharded 900 $PT tests/test_gpu_sharded.py
for pr in ${PROBES_LIST:-}; do
  set -- $pr
  GCR_PROBE=$1 GCR_VERIFY_CHAIN=$2 timeout -k 10 120 python bench.py --steps 2000 --warmup 20 --cpu-seconds 0 --no-latency --no-hbm-probe > $D/probe_$1_$2.json 2>/dev/null || { echo "probe $pr failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$D/probe_$1_$2.json').read().strip().splitlines()[-1]); print('probe $1 chain $2: kernel', round(d['roofline']['avg_kernel_ms']*1e3,1), 'us step', round(d['ms_per_step']*1e3,1))"
done
echo "session done"
