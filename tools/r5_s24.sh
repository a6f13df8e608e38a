export OUT=gpurun_out/r5_s24
STEPS="suite ktrace trace lat" TESTS="tests/test_gpu_lo_approx.py tests/test_gpu_parity.py tests/test_gpu_exact.py -m gpu" KTRACE_ENVS="GCR_LO_APPROX_FUSE=1" LAT_SETS="fuse: nofuse:GCR_LO_APPROX_FUSE=0" bash tools/r5.sh
