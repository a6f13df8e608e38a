#!/bin/bash
# F / H band session: correspondence-scorer parity, then the F and H bench
# lines with the feature-major scorer and with the split scorer beside it.
set -u
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -c 1500 "gpurun_out/$name.log"; echo
  case $rc in 0|1) return 0 ;; *) echo "fatal rc=$rc"; exit $rc ;; esac
}
step tests_geo 600 python -u -m pytest tests/test_gpu_geo_band.py tests/test_fundamental.py tests/test_homography.py tests/test_gpu_bench_config.py -m gpu -x -q -rf --timeout 300 --timeout-method thread
step benchf 300 python bench.py --workload f --cpu-seconds 0 --no-hbm-probe
step benchf_split 300 env GCR_SCORER=split python bench.py --workload f --cpu-seconds 0 --no-hbm-probe
step benchh 300 python bench.py --workload h --cpu-seconds 0 --no-hbm-probe
step benchh_split 300 env GCR_SCORER=split python bench.py --workload h --cpu-seconds 0 --no-hbm-probe
echo "session done"
