#!/bin/bash
# End-of-round-3 measurement, second pass (LO-winner reuse in the final refit): GPU suite, smoke(), the
# driver's bench line (M2), F / H / M1 lines, strong N=1, configs[4] batch
# (default lambda and 0), rocprofv3 --stats + PMC passes for M2 and F.
set -u
D=gpurun_out/r3_final2
mkdir -p $D
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$D/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n ${TAILN:-3} "$D/$name.log" | cut -c1-400
    [ $rc -eq 0 ] || { echo "fatal rc=$rc, stopping"; exit $rc; }
}
run reuse_tests 300 python -u -m pytest tests/test_gpu_refit_reuse.py -x -q --timeout 120 --timeout-method thread
run tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
run lat_m2 300 python -u tools/lat_ab.py --workload m2 --reps 5 reuse: noreuse:GCR_LO_REUSE=0
run lat_m1 300 python -u tools/lat_ab.py --workload m1 --reps 4 reuse: noreuse:GCR_LO_REUSE=0
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_m2 400 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_f 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe
run bench_h 300 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe
run bench_m1 300 python bench.py --workload m1 --cpu-seconds 0 --no-hbm-probe
run strong1 300 python bench.py --mode strong --steps 16 --warmup 2
run batch_def 400 python bench.py --workload batch --cpu-seconds 0 --no-hbm-probe
run batch_l0 400 python bench.py --workload batch --batch-lambda 0 --cpu-seconds 0 --no-hbm-probe
WL=m2 TAG=r3_final2/m2 STATS=1 PMC=1 bash tools/r3_measure.sh || exit 1
WL=f TAG=r3_final2/f STATS=1 PMC=1 bash tools/r3_measure.sh || exit 1
WL=h TAG=r3_final2/h STATS=1 PMC=1 bash tools/r3_measure.sh || exit 1
echo "session r3_final2 done"
