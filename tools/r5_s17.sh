export OUT=gpurun_out/r5_s17
STEPS="trace" bash tools/r5.sh
