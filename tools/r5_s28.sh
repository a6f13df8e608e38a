export OUT=gpurun_out/r5_s28
mkdir -p $OUT
for q in 8 16; do for c in 8 12 16; do GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --workload batch --cpu-seconds 0 --concurrency $c > $OUT/batch_q${q}_$c.log 2>&1 || exit 1; tail -1 $OUT/batch_q${q}_$c.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('queues $q conc $c', d['config']['problems_per_s'])"; done; done
