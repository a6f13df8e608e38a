export OUT=gpurun_out/r5_s29
mkdir -p $OUT
GCR_LIB=libgcr_stamps.so timeout -k 10 200 python -u tools/stamp_probe.py --workload m2 > $OUT/stamps.log 2>&1; cat $OUT/stamps.log | tail -40
