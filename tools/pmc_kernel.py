#!/usr/bin/env python3
"""Per-kernel PMC summary of a rocprofv3 --pmc run (run_counter_collection.csv):
mean counter value per dispatch for kernels whose name matches a pattern.
usage: pmc_kernel.py COUNTER_COLLECTION.csv [--match k_sift_gram]"""
import argparse
import csv
import re
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--match", default="")
a = ap.parse_args()
vals = {}
for r in csv.DictReader(open(a.csv)):
    name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("gcr::(anonymous namespace)::", ""))
    if a.match and not re.search(a.match, name):
        continue
    key = (name, r["Counter_Name"])
    vals.setdefault(key, {}).setdefault(r["Dispatch_Id"], 0.0)
    vals[key][r["Dispatch_Id"]] += float(r["Counter_Value"])
for (name, ctr), d in sorted(vals.items()):
    v = list(d.values())
    print(f"  {name[:40]:40s} {ctr:28s} n={len(v):4d} mean {statistics.mean(v):14.1f}")
