export OUT=gpurun_out/r5_s30
STEPS="suite trace lat" TESTS="tests/test_gpu_lo_approx.py tests/test_gpu_parity.py tests/test_gpu_exact.py tests/test_gpu_fold.py tests/test_gpu_refit_reuse.py -m gpu" bash tools/r5.sh
