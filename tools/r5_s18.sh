export OUT=gpurun_out/r5_s18
STEPS="suite trace" TESTS="tests/test_gpu_parity.py tests/test_frozen_pin.py tests/test_gpu_lo_approx.py -m gpu" bash tools/r5.sh
