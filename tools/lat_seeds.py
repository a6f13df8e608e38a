#!/usr/bin/env python3
"""Per-seed wall time to 0.99 confidence (bench.py's latency calls, seeds
100..110) under two settings, interleaved: time, iterations, chunks (slots),
LO / graph-cut rounds.  usage: lat_seeds.py [--workload m2] [--reps 3] NAME:ENV=V ..."""
import argparse
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "graph-cut-ransac_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import bench  # noqa: E402
import lat_ab  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="m2")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("settings", nargs="+")
a = ap.parse_args()
f0, f1, thr0, thr1, solver, _ = bench.workload_problem(a.workload, 20251121)
sets = []
for s in a.settings:
    name, _, env = s.partition(":")
    sets.append((name, dict(kv.split("=", 1) for kv in env.split(",") if kv)))
lat_ab.call(solver, f0, f1, thr0, thr1, 99)
res = {}
for rep in range(a.reps):
    for seed in range(100, 111):
        for name, env in sets:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            t = time.perf_counter()
            out = lat_ab.call(solver, f0, f1, thr0, thr1, seed)
            ms = (time.perf_counter() - t) * 1e3
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            st = out[-1]
            res.setdefault((name, seed), []).append((ms, st["iteration_number"], st["slots"],
                                                     st["local_optimization_number"], st["graph_cut_number"],
                                                     st.get("prefetched_chunks", 0),
                                                     {k: st.get(k, 0.0) for k in ("ms_score", "ms_replay", "ms_lo",
                                                                                  "ms_lo_fit", "ms_lo_score",
                                                                                  "ms_refit", "lo_models")}))
for seed in range(100, 111):
    row = [f"seed {seed}"]
    for name, _ in sets:
        r = res[(name, seed)]
        ph = " ".join(f"{k[3:] if k.startswith('ms_') else k}={statistics.median(x[6][k] for x in r):.3f}"
                      for k in r[0][6])
        row.append(f"{name}: {statistics.median(x[0] for x in r):6.3f} ms it {r[0][1]:5d} slots {r[0][2]:6d} "
                   f"lo {r[0][3]} gc {r[0][4]} pf {r[0][5]} {ph}")
    print("  |  ".join(row))
for name, _ in sets:
    per = [statistics.median(x[0] for x in res[(name, seed)]) for seed in range(100, 111)]
    print(f"{name}: median over seeds {statistics.median(per):.3f} ms, worst {max(per):.3f} ms")
