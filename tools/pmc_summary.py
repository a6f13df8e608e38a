#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes: mean counter value per dispatch, per kernel.

usage: tools/pmc_summary.py gpurun_out/pmc > profiles/<name>.csv

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


def main(root):
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


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
