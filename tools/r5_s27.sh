export OUT=gpurun_out/r5_s27
mkdir -p $OUT
for c in 8 12 16; do timeout -k 10 300 python -u bench.py --workload batch --cpu-seconds 0 --concurrency $c > $OUT/batch_$c.log 2>&1 || exit 1; tail -1 $OUT/batch_$c.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('conc $c', d['config']['problems_per_s'])"; done
for t in 4 8; do GCR_HOST_THREADS=$t timeout -k 10 300 python -u bench.py --workload batch --cpu-seconds 0 --concurrency 16 > $OUT/batch_t$t.log 2>&1 || exit 1; tail -1 $OUT/batch_t$t.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('conc 16 pool $t', d['config']['problems_per_s'])"; done
