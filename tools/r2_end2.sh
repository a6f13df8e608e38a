#!/bin/bash
# Round-2 end-of-round measurement session, second pass (after deferred
# selection; first pass after the widening generator and
# the homography pre-band): GPU suite, the driver's bench line (with CPU
# baseline and latency leg), the other workloads, strong scaling on one GPU,
# the rocprofv3 kernel stats of the M2 line and PMC passes (SQ, FETCH, WRITE)
# for the M2 / H / F scorers.  Every GPU step under its own time limit; a
# crash, abort or timeout ends the session.
set -u
mkdir -p gpurun_out/end2
O=gpurun_out/end2
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -c 400 "$O/$name.log"; echo
  case $rc in 0|1) return 0 ;; *) echo "fatal rc=$rc"; exit $rc ;; esac
}
step tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
step bench_m2 400 python bench.py --gpus 1 --steps 20 --warmup 5
step bench_m1 300 python bench.py --workload m1 --cpu-seconds 0 --no-hbm-probe
step bench_h 300 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe
step bench_f 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe
step bench_batch 300 python bench.py --workload batch --cpu-seconds 0 --no-hbm-probe
step strong1 300 python bench.py --mode strong --steps 16 --warmup 4 --cpu-seconds 0 --no-hbm-probe
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step prof_m2 300 rocprofv3 --kernel-trace --stats -d $O/prof_m2 -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-hbm-probe
for w in m2 h f; do
  i=0
  while IFS= read -r ctrs; do
    [ -z "$ctrs" ] && continue; i=$((i+1))
    step pmc_${w}_$i 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $O/pmc_$w/pass$i -o run -- python3 bench.py --workload $w --steps 20 --warmup 2 --cpu-seconds 0 --no-latency --no-hbm-probe
  done < tools/pmc_sets_r2.txt
done
echo "session done"
