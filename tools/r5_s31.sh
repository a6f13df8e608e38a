export OUT=gpurun_out/r5_s31
STEPS="trace" bash tools/r5.sh
