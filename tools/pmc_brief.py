"""Mean SQ counters per kernel of a tools/pmc_session.sh run (CLI summary)."""
import collections
import csv
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ("pass1", "pass2"):
    try:
        rows = list(csv.DictReader(open(f"{d}/{p}/run_counter_collection.csv")))
    except OSError:
        continue
    for r in rows:
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for k, v in agg.items():
    if pat in k:
        m = {c: sum(x) / len(x) for c, x in v.items()}
        w = m.get("SQ_WAVES", 1)
        print(k[:70])
        print("  " + "  ".join(f"{c}={x:.4g}" for c, x in sorted(m.items())))
        if "SQ_INSTS_VALU" in m:
            print(f"  VALU/wave={m['SQ_INSTS_VALU'] / w:.0f} SALU/wave={m.get('SQ_INSTS_SALU', 0) / w:.0f} "
                  f"LDS/wave={m.get('SQ_INSTS_LDS', 0) / w:.0f} issue_us={m['SQ_INSTS_VALU'] * 4 / 1024 / 2400:.1f}")
