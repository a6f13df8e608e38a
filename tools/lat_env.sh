set -u
mkdir -p gpurun_out
for v in default interrupt0; do
  if [ $v = interrupt0 ]; then export HSA_ENABLE_INTERRUPT=0; fi
  timeout -k 10 300 python tools/latency_probe.py --reps 10 > gpurun_out/latency_$v.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/latency_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/latency_$v.log)"
  timeout -k 10 300 python bench.py --workload h --cpu-seconds 0 --steps 500 --warmup 50 > gpurun_out/bh_$v.log 2>&1 || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*\|"ms_median": [0-9.]*' gpurun_out/bh_$v.log | tr '\n' ' ')"
done
