#!/bin/bash
# PMC passes (each its own rocprofv3 run, counters + kernel trace only).
set -u
D="${PMC_DIR:-gpurun_out/pmc}"
mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ARGS="${BENCH_ARGS:---steps 3 --warmup 1 --cpu-seconds 0 --no-latency --slots 65536}"
timeout -k 10 120 rocprofv3 -L > "$D"/counters_list.txt 2>&1 || true
i=0
while IFS= read -r ctrs; do
  [ -z "$ctrs" ] && continue; i=$((i+1))
  echo "=== pass$i: $ctrs"
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$D"/pass$i -o run -- python3 bench.py $ARGS > "$D"/pass$i.log 2>&1
  rc=$?; echo "rc=$rc"; tail -3 "$D"/pass$i.log
  case $rc in 0) ;; *) echo "stopping"; exit $rc ;; esac
done < "${PMC_FILE:-tools/pmc_sets.txt}"
