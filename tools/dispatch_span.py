#!/usr/bin/env python3
"""Throughput time per dispatch of one kernel from a rocprofv3 kernel trace
(run_kernel_trace.csv): the dispatches are split into bursts at gaps longer
than --split us (bench.py's warm-up, extra warm-up and timed calls), and per
burst it prints the count, the span from the first start to the last end, that
span over the count (the per-launch time bench.py's overlapped launches
report as avg_kernel_ms), the mean dispatch duration and the mean number of
dispatches in flight.  usage: dispatch_span.py TRACE.csv [--kernel k_score_fm] [--split 200]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--kernel", default="k_score_fm")
ap.add_argument("--split", type=float, default=200.0)
a = ap.parse_args()
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
              for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"])
bursts, cur, last_end = [], [], None
for s0, e0 in rows:
    if cur and (s0 - last_end) / 1e3 > a.split:
        bursts.append(cur)
        cur = []
    cur.append((s0, e0))
    last_end = e0 if last_end is None or not cur[:-1] else max(last_end, e0)
bursts.append(cur)
print(f"kernel {a.kernel}: {len(rows)} dispatches in {len(bursts)} bursts (gap > {a.split} us)")
for b in bursts:
    span = (max(e for _, e in b) - b[0][0]) / 1e3
    dur = sum(e - s for s, e in b) / 1e3
    print(f"  {len(b):6d} dispatches  span {span:10.1f} us  span/dispatch {span / len(b):8.2f} us  "
          f"mean dispatch {dur / len(b):8.2f} us  in flight {dur / span:5.2f}")
