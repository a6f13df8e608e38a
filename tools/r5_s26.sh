export OUT=gpurun_out/r5_s26
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --workload batch --cpu-seconds 0 > $OUT/batch.log 2>&1 && tail -1 $OUT/batch.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('batch',d['value'],d['unit'],d.get('ms_per_step'))" && STEPS="benchf" bash tools/r5.sh
