#!/bin/bash
# configs[4] batch: HIP hardware queues per process (GPU_MAX_HW_QUEUES, the
# box default 4) x problems in flight (--concurrency).  Each problem context
# has two streams, so 8 problems put 16 streams on the process's queues.
set -u
O=gpurun_out/bhwq
mkdir -p $O
for cfg in 4:8 8:8 16:8 16:16 24:12; do
  q=${cfg%%:*}; c=${cfg##*:}
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --workload batch --concurrency $c --cpu-seconds 0 --no-hbm-probe > $O/b_q${q}_c$c.log 2>&1 || { tail -20 $O/b_q${q}_c$c.log; exit 1; }
done
echo "session done"
