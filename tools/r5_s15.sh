export OUT=gpurun_out/r5_s15
STEPS="suite trace lat" TESTS="tests/test_gpu_lo_approx.py tests/test_gpu_score_guard.py tests/test_gpu_exact.py" LAT_SETS="apx: noapx:GCR_LO_APPROX=0" bash tools/r5.sh
