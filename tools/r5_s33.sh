export OUT=gpurun_out/r5_s33
STEPS="suite trace lat" TESTS="tests/test_gpu_parity.py tests/test_gpu_exact.py tests/test_gpu_lo_approx.py tests/test_gpu_sharded.py -m gpu" bash tools/r5.sh
