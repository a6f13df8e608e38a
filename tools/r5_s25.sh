export OUT=gpurun_out/r5_s25
STEPS="valu" bash tools/r5.sh && PMC_DIR=gpurun_out/r5_s25/pmc PMC_FILE=tools/pmc_sets_r4.txt bash tools/pmc_session.sh && STEPS="stats" BENCH_ARGS="--steps 200 --warmup 20 --no-latency" OUT=gpurun_out/r5_s25 bash tools/r5.sh
