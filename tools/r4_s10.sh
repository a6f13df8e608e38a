set -u
O=gpurun_out/r4_s10; mkdir -p $O
for set in "base:" "nofold:GCR_PROBE=256" "noresid:GCR_PROBE=512" "neither:GCR_PROBE=768" "seq:GCR_LO_FOLD=seq"; do
  tag=${set%%:*}; env=${set#*:}
  timeout -k 10 120 env TAG=$tag $env python -u tools/lo_probe.py >> $O/probe.log 2>&1 || { echo "rc=$?"; exit 1; }
done
cat $O/probe.log
timeout -k 10 120 python -u tools/fold_bench.py
