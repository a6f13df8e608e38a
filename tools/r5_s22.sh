export OUT=gpurun_out/r5_s22
STEPS="suite ktrace trace" TESTS="tests/test_gpu_parity.py tests/test_frozen_pin.py -m gpu" KTRACE_ENVS="GCR_GRAM_BATCH=1 GCR_GRAM_BATCH=2" bash tools/r5.sh
