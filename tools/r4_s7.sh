set -u
O=gpurun_out/r4_s7; mkdir -p $O
run() { local n=$1 to=$2; shift 2; echo "=== $n"; timeout -k 10 $to "$@" > $O/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -n 9 $O/$n.log; case $rc in 0|1) ;; *) exit $rc;; esac; }
run foldtest 300 python -u -m pytest tests/test_gpu_fold.py -q -x --timeout 120 --timeout-method thread
run foldbench 120 python -u tools/fold_bench.py
run lat 300 python -u tools/lat_ab.py --workload m2 --reps 4 base: wide:GCR_LO_FOLD=wide
