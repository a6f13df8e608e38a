export OUT=gpurun_out/r5_s35
mkdir -p $OUT
for rep in 1 2; do for pr in 0 1024; do GCR_PROBE=$pr timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 --no-latency --cpu-seconds 0 --no-hbm-probe > $OUT/b_${pr}_$rep.log 2>&1 || exit 1; tail -1 $OUT/b_${pr}_$rep.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('probe $pr rep $rep', d['value'], d['ms_per_step'], d['roofline']['avg_kernel_ms'])"; done; done
STEPS="suite" TESTS="tests/test_gpu_parity.py -m gpu" bash tools/r5.sh
