#!/usr/bin/env python3
"""Timeline of one call from a rocprofv3 kernel trace (run_kernel_trace.csv):
every dispatch's start, duration and the gap since the previous one ended,
for the calls of tools/lat_seeds.py (split by gaps > --split us).  Shows
where a short call's wall time goes between kernels (host work, launch and
completion latency).  usage: trace_gaps.py TRACE.csv [--call K] [--split 300] [--summary]"""
import argparse
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--call", type=int, default=3)
ap.add_argument("--split", type=float, default=300.0)
ap.add_argument("--summary", action="store_true", help="per-kernel count / median / mean duration instead")
a = ap.parse_args()
rows = []
for r in csv.DictReader(open(a.trace)):
    name = r["Kernel_Name"].replace("void ", "").replace("gcr::(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r["Queue_Id"]))
rows.sort()
if a.summary:
    import statistics
    by = {}
    for s0, e0, n, _ in rows:
        by.setdefault(n, []).append((e0 - s0) / 1e3)
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n[:48]:48s} n={len(v):5d} median {statistics.median(v):8.1f} us  mean {statistics.mean(v):8.1f}")
    raise SystemExit(0)
calls, cur = [], []
for r in rows:
    if cur and (r[0] - cur[-1][1]) / 1e3 > a.split:
        calls.append(cur)
        cur = []
    cur.append(r)
calls.append(cur)
print(f"{len(calls)} calls; call {a.call}:")
c = calls[a.call]
t0, prev = c[0][0], c[0][0]
for s, e, n, q in c:
    print(f"  t={(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:7.1f}  gap {(s - prev) / 1e3:7.1f}  q{q}  {n}")
    prev = max(prev, e)
print(f"  span {(prev - t0) / 1e3:.1f} us")
