set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for w in h f; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 100 --warmup 10 --cpu-seconds 0 --no-latency > gpurun_out/prof_$w.log 2>&1 || { echo "prof $w failed rc=$?"; exit 1; }
done
find gpurun_out -name "*kernel_stats.csv" | head
