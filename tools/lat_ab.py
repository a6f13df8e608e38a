#!/usr/bin/env python3
"""Latency A/B in one process: the bench's wall-time-to-0.99 call (bench.py
latency leg: same problems, seeds 100..110) under several environment
settings, interleaved rep by rep so clock and cache state hit every setting
alike.  Prints per setting the median over all calls and the median phase
breakdown.

usage: python tools/lat_ab.py --workload f --reps 5 base: nospec:GCR_SPECULATE=0 seq:GCR_LO_FOLD=seq,GCR_X=1
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "graph-cut-ransac_amd"))

import bench  # noqa: E402
import pygcransac  # noqa: E402
from pygcransac import _native as N  # noqa: E402

KEYS = ("ms_setup", "ms_score", "ms_replay", "ms_lo", "ms_lo_lists", "ms_lo_fit", "ms_lo_score", "ms_refit_fit", "ms_exact",
        "exact_models", "exact_pairs",
        "ms_refit", "ms_total")


def call(solver, f0, f1, thr0, thr1, seed):
    if solver == N.SOLVER_FUNDAMENTAL7:
        return pygcransac.findFundamentalMatrix(f0, 960, 1280, 960, 1280, threshold=thr0, conf=0.99, min_iters=0,
                                                max_iters=10**7, seed=seed, return_stats=True)
    if solver == N.SOLVER_HOMOGRAPHY4:
        return pygcransac.findHomography(f0, 960, 1280, 960, 1280, threshold=thr0, conf=0.99, min_iters=0,
                                         max_iters=10**7, seed=seed, return_stats=True)
    if solver == N.SOLVER_SIFT22:
        return pygcransac.findRectifyingHomographySIFT(f0, f1, thr0, thr1, 0.0, 0, 10**7, 50, seed=seed,
                                                      confidence=0.99, return_stats=True)
    return pygcransac.findRectifyingHomographyScaleOnly(f0, thr0, 0.0, 0, 10**7, 50, seed=seed, confidence=0.99,
                                                        return_stats=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="m2", choices=["m2", "m1", "h", "f"])
    ap.add_argument("--reps", type=int, default=3, help="passes over the 11 bench seeds")
    ap.add_argument("--json", default=None)
    ap.add_argument("settings", nargs="+", help="name:VAR=VAL,VAR=VAL (empty after ':' = unchanged env)")
    a = ap.parse_args()
    f0, f1, thr0, thr1, solver, text = bench.workload_problem(a.workload, 20251121)
    sets = []
    for s in a.settings:
        name, _, kv = s.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        sets.append((name, env))
    for _ in range(3):                              # warm-up (context, pinned pools, clocks)
        call(solver, f0, f1, thr0, thr1, 99)
    res = {name: {"ms": [], "stats": []} for name, _ in sets}
    for rep in range(a.reps):
        for si in range(11):
            order = sets[(rep + si) % len(sets):] + sets[:(rep + si) % len(sets)]
            for name, env in order:
                old = {k: os.environ.get(k) for k in env}
                os.environ.update(env)
                t0 = time.perf_counter()
                out = call(solver, f0, f1, thr0, thr1, 100 + si)
                res[name]["ms"].append((time.perf_counter() - t0) * 1e3)
                res[name]["stats"].append(out[-1])
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
    summary = {}
    for name, _ in sets:
        ms = res[name]["ms"]
        bd = {k: statistics.median(s[k] for s in res[name]["stats"]) for k in KEYS}
        summary[name] = {"median_ms": statistics.median(ms), "mean_ms": statistics.fmean(ms), "n": len(ms),
                         "breakdown_median": bd}
        print(f"{a.workload} {name:>10}: median {statistics.median(ms):.3f} ms  mean {statistics.fmean(ms):.3f}  " +
              " ".join(f"{k[3:] if k.startswith('ms_') else k}={v:.3f}" for k, v in bd.items()), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"workload": text, "settings": dict(sets), "summary": summary,
                       "ms_all": {n: res[n]["ms"] for n in res}}, f, indent=1)


if __name__ == "__main__":
    main()
