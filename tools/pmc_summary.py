#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes: mean counter value per dispatch, per kernel.

usage: tools/pmc_summary.py gpurun_out/pmc [--slots N --traffic-json profiles/pmc_traffic.json
                                           --stats <rocprofv3 kernel_stats.csv of the same command>]
                                           > profiles/<name>.csv

Each traffic-json entry records the kernel build it was collected from
(`kernel_build_id`, read from the bench JSON line the passes printed), so
bench.py never reuses counters of an older build of the kernels.

FETCH_SIZE is reported as measured (KiB) and corrected: MI355X_MICROARCH.md's
HBM section notes gfx950 under-reports wide streaming reads by 2x, so the
corrected HBM-read bytes column doubles it.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+<[^>]*>)", name)
    return m.group(1) if m else name[:60]


def build_id_of(root):
    """kernel_build_id of the bench line printed by the passes (all must agree)."""
    import json
    ids = set()
    for path in glob.glob(os.path.join(root, "pass*.log")):
        with open(path) as f:
            for ln in f:
                if ln.startswith("{") and "kernel_build_id" in ln:
                    try:
                        ids.add(json.loads(ln)["roofline"]["kernel_build_id"])
                    except (ValueError, KeyError, TypeError):
                        pass
    if len(ids) != 1:
        raise SystemExit(f"expected one kernel_build_id in {root}/pass*.log, found {sorted(ids)}")
    return ids.pop()


def stats_avg_ms(stats_csv):
    """kernel -> average duration (ms) from a rocprofv3 --stats kernel_stats.csv."""
    out = {}
    if stats_csv:
        with open(stats_csv) as f:
            for row in csv.DictReader(f):
                out[short(row["Name"])] = float(row["AverageNs"]) / 1e6
    return out


def main(root, slots=None, traffic_json=None, stats_csv=None):
    vals = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(root, "pass*", "*counter_collection.csv"))):
        with open(path) as f:
            for row in csv.DictReader(f):
                vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "counter", "dispatches", "mean_per_dispatch"])
    for k in sorted(vals):
        for c in sorted(vals[k]):
            v = vals[k][c]
            w.writerow([k, c, len(v), f"{sum(v) / len(v):.6g}"])
        if "FETCH_SIZE" in vals[k]:
            v = vals[k]["FETCH_SIZE"]
            w.writerow([k, "HBM_READ_BYTES_corrected(2*FETCH_SIZE*1024)", len(v), f"{2048 * sum(v) / len(v):.6g}"])
    if traffic_json and slots:
        import json
        try:
            with open(traffic_json) as f:
                table = json.load(f)
        except (OSError, ValueError):
            table = {}
        bid = build_id_of(root)
        avg = stats_avg_ms(stats_csv)
        for k in vals:
            if "FETCH_SIZE" not in vals[k] or not k.startswith("k_score"):
                continue
            rd = 2048 * sum(vals[k]["FETCH_SIZE"]) / len(vals[k]["FETCH_SIZE"])
            wr = vals[k].get("WRITE_SIZE")
            wrb = 1024 * sum(wr) / len(wr) if wr else 0.0
            ent = {"hbm_bytes_per_launch": rd + wrb, "read_bytes": rd, "write_bytes": wrb,
                   "source": os.path.normpath(root), "kernel_build_id": bid}
            if k in avg:
                ent["rocprof_avg_ms"] = avg[k]
            # VALU view (bench.py "valu", "roofline.valu_issue"): instructions
            # issued per class, active VALU quad-cycles, waits -- every SQ_
            # counter collected for this kernel (mean per launch)
            for c in sorted(vals[k]):
                if c.startswith("SQ_"):
                    ent[c] = sum(vals[k][c]) / len(vals[k][c])
            table[f"{k}@{slots}"] = ent
        with open(traffic_json, "w") as f:
            json.dump(table, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--slots", type=int)
    ap.add_argument("--traffic-json")
    ap.add_argument("--stats")
    a = ap.parse_args()
    main(a.root, a.slots, a.traffic_json, a.stats)
