#!/bin/bash
set -u
D=gpurun_out/${TAG:-r3_s9}
mkdir -p $D
timeout -k 10 300 python -u -m pytest -s tests/test_gpu_lo_fold.py "tests/test_gpu_parity.py::test_small_batch_scorer_matches_oracle_bitwise" "tests/test_gpu_parity.py::test_full_size_m1_and_m2_match_oracle_and_ground_truth" -q -x --timeout 120 --timeout-method thread > $D/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 $D/tests.log
[ $rc -eq 0 ] || exit $rc
GCR_LO_FOLD=wave timeout -k 10 300 python -u -m pytest tests/test_gpu_lo_fold.py -q -x --timeout 120 --timeout-method thread > $D/tests_wave.log 2>&1; echo "wave rc=$?"; tail -1 $D/tests_wave.log
WL=m2 TAG=r3_s9 bash tools/r3_s8.sh
