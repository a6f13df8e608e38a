#!/bin/bash
set -u
D=gpurun_out/${TAG:-r3_s7}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_lo_fold.py "tests/test_gpu_parity.py::test_small_batch_scorer_matches_oracle_bitwise" -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1; echo "rc=$?"
tail -15 $D/tests.log
GCR_LO_FOLD=seq timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_full_size_m1_and_m2_match_oracle_and_ground_truth" -q --timeout 120 --timeout-method thread > $D/full_seq.log 2>&1; echo "full seq rc=$?"; tail -2 $D/full_seq.log
