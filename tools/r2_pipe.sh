#!/bin/bash
# correspondence batch pipeline: parity, then F / H bench lines pipe on / off
set -u
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -c 600 "gpurun_out/$name.log"; echo
  case $rc in 0) return 0 ;; *) echo "fatal rc=$rc"; exit $rc ;; esac
}
step tests_pipe 600 python -u -m pytest tests/test_gpu_bench_config.py tests/test_fundamental.py tests/test_homography.py tests/test_gpu_geo_band.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "correspondence or pipelined or verify or band or score or generate"
step benchf 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe --no-latency
step benchf_nopipe 300 env GCR_VERIFY_PIPE=0 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe --no-latency
step benchh 300 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe --no-latency
step benchh_nopipe 300 env GCR_VERIFY_PIPE=0 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe --no-latency
echo "session done"
