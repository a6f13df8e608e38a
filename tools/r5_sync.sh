#!/bin/bash
# host wake-up latency of HIP's wait policies (tools/micro/sync_latency.hip)
set -u
for m in auto spin yield blocking; do echo "== $m"; timeout -k 5 60 tools/micro/sync_latency.bin $m || exit 1; done
for t in 10 50 1000; do echo "== ROC_ACTIVE_WAIT_TIMEOUT=$t"; ROC_ACTIVE_WAIT_TIMEOUT=$t timeout -k 5 60 tools/micro/sync_latency.bin || exit 1; done
