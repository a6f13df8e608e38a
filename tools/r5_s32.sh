export OUT=gpurun_out/r5_s32
STEPS="suite trace lat" bash tools/r5.sh
