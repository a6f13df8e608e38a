export OUT=gpurun_out/r5_s19
STEPS="ktrace trace" KTRACE_ENVS="GCR_GRAM_BATCH=1 GCR_GRAM_BATCH=2 GCR_GRAM_BATCH=4" bash tools/r5.sh
