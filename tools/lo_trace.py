#!/usr/bin/env python3
"""Host timeline of the LO rounds of a few latency calls (GCR_LO_TRACE=1 is
printed by the engine to stderr; this runs bench.py's latency workload for
seeds 100..104 and summarises the per-round phase durations).
usage: GCR_LO_TRACE=1 lo_trace.py 2> trace.txt; lo_trace.py --parse trace.txt"""
import os
import re
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2 and sys.argv[1] == "--parse":
    for label in ("LO:", "RUN:", "SETUP:"):
        deltas = {}
        for ln in open(sys.argv[2]):
            if not ln.startswith("gcr " + label):
                continue
            toks = ln.split()[2:]
            ev = [(toks[i], float(toks[i + 1])) for i in range(0, len(toks), 2)]
            for (a, ta), (b, tb) in zip(ev, ev[1:]):
                deltas.setdefault(f"{a}->{b}", []).append(tb - ta)
        if deltas:
            print(label)
        for k, v in sorted(deltas.items(), key=lambda kv: -statistics.median(kv[1])):
            print(f"  {k:24s} n={len(v):4d} median {statistics.median(v):7.1f} us  mean {statistics.mean(v):7.1f}")
    sys.exit(0)
sys.path[:0] = [REPO, os.path.join(REPO, "graph-cut-ransac_amd"), os.path.join(REPO, "tools")]
import bench  # noqa: E402
import lat_ab  # noqa: E402

f0, f1, thr0, thr1, solver, _ = bench.workload_problem(sys.argv[1] if len(sys.argv) > 1 else "m2", 20251121)
lat_ab.call(solver, f0, f1, thr0, thr1, 99)
for rep in range(3):
    for seed in range(100, 111):
        lat_ab.call(solver, f0, f1, thr0, thr1, seed)
print("done", flush=True)
