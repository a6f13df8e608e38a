#!/bin/bash
# round-4 session 28: asynchronous feature upload -- GPU suite, latency A/B against the previous engine
set -u
O=gpurun_out/r4_s28; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 300 python -u tools/lat_ab.py --workload m2 --reps 7 async: sync:GCR_UPLOAD_SYNC=1 > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
cat $O/lat.log
