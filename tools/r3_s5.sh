#!/bin/bash
# GPU suite + latency A/B of the LO fold (GCR_LO_FOLD=seq), the speculative
# chunk issue (GCR_SPECULATE=0) and the chunk cap (GCR_CHUNK_CAP=0).
set -u
D=gpurun_out/${TAG:-r3_s5}
mkdir -p $D
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$D/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n ${TAILN:-3} "$D/$name.log" | cut -c1-600
    case $rc in 0|1|5) return 0 ;; *) echo "fatal rc=$rc, stopping"; exit $rc ;; esac
}
lat() {  # name workload [env...]
    local name=$1 wl=$2; shift 2
    run "$name" 300 env "$@" python bench.py --workload $wl --steps 200 --warmup 20 --cpu-seconds 0 --no-hbm-probe
    python3 - "$D/$name.log" "$name" <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d["wall_time_to_0.99_confidence"]; b = w["ms_breakdown"]
print(f"LAT {sys.argv[2]}: median {w['ms_median']:.3f} ms  " + " ".join(f"{k[3:]}={v:.3f}" for k, v in b.items() if k.startswith("ms_")))
P
}
[ -n "${NOTESTS:-}" ] || run tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
for wl in m2 h f; do
  lat lat_${wl} $wl GCR_X=1
  lat lat_${wl}_seqfold $wl GCR_LO_FOLD=seq
done
lat lat_f_nospec f GCR_SPECULATE=0
lat lat_f_nocap f GCR_CHUNK_CAP=0
lat lat_f_neither f GCR_SPECULATE=0 GCR_CHUNK_CAP=0
echo "session done"
