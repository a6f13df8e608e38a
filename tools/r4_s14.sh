#!/bin/bash
# round-4 session 14: split small-batch scorer (k_lo_resid + k_lo_fold) --
# device fold / small-scorer tests, parity suite, latency A/B split vs
# k_lo_chain, kernel trace of the latency call
set -u
O=gpurun_out/r4_s14; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/lat_ab.py --workload m2 --reps 5 base: nosplit:GCR_LO_SPLIT=0 > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
cat $O/lat.log
timeout -k 10 300 python -u tools/lat_ab.py --workload f --reps 3 base: nosplit:GCR_LO_SPLIT=0 > $O/lat_f.log 2>&1 || { tail -20 $O/lat_f.log; exit 1; }
cat $O/lat_f.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/latency_probe.py --reps 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -12 $O/kernel_stats.csv
timeout -k 10 120 python -u tools/fold_bench.py > $O/fold_bench.log 2>&1 || { cat $O/fold_bench.log; exit 1; }
cat $O/fold_bench.log
