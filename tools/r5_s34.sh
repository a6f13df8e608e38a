export OUT=gpurun_out/r5_s34
STEPS="suite" TESTS="tests/test_gpu_setup.py tests/test_gpu_summary.py -m gpu" bash tools/r5.sh
