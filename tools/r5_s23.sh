export OUT=gpurun_out/r5_s23
STEPS="suite trace lat" bash tools/r5.sh
