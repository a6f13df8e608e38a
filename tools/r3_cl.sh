set -u
D=gpurun_out/r3_cl
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_refit_reuse.py -x -q --timeout 300 --timeout-method thread > $D/cl_tests.log 2>&1; rc=$?
echo "cl tests rc=$rc"; tail -2 $D/cl_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $D/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lat_seeds.py --workload m2 --reps 3 base: nocl:GCR_CHUNK_LISTS=0 > $D/seeds_m2.log 2>&1 || exit 1
tail -11 $D/seeds_m2.log
timeout -k 10 300 python -u tools/lat_ab.py --workload m2 --reps 5 cl: nocl:GCR_CHUNK_LISTS=0 > $D/lat_m2.log 2>&1 || exit 1
tail -2 $D/lat_m2.log
timeout -k 10 300 python -u tools/lat_ab.py --workload m1 --reps 4 cl: nocl:GCR_CHUNK_LISTS=0 > $D/lat_m1.log 2>&1 || exit 1
tail -2 $D/lat_m1.log
