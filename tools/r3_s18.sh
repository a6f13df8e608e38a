#!/bin/bash
# Re-entry check of the round-3 build: full GPU suite, smoke(), the default
# (driver-shaped) bench line, then rocprofv3 --stats + PMC passes for M2 and F
# so profiles/pmc_traffic.json matches this kernel build.
set -u
T=${TAG:-r3_s18}
D=gpurun_out/$T
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $D/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $D/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $D/bench.log 2> $D/bench.err || { echo "bench failed"; tail -5 $D/bench.err; exit 1; }
tail -c 600 $D/bench.log
WL=m2 TAG=$T/m2 STATS=1 PMC=1 bash tools/r3_measure.sh || exit 1
WL=f TAG=$T/f STATS=1 PMC=1 bash tools/r3_measure.sh || exit 1
echo "session $T done"
