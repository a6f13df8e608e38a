#!/usr/bin/env python3
"""Repeat the configs[4] batch (bench.batch_problems, gcr_solve_batch with 8
host threads) and require every repetition to equal the first bit for bit:
a stress test of the concurrent host paths (host pool, pipelined LO trial
scoring, completion-flag waits).  usage: stress_batch.py [reps] [n]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "graph-cut-ransac_amd")]
import bench  # noqa: E402
from pygcransac import distributed as D  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
problems = bench.batch_problems(n)
solve = D.batch_solver(0, 8)


def digest(out):
    return [(None if r["H"] is None else np.asarray(r["H"]).tobytes(),
             tuple(np.asarray(m, dtype=bool).tobytes() for m in r["masks"]), r["stats"]["iteration_number"])
            for r in out]


ref = None
for k in range(reps):
    t = time.perf_counter()
    d = digest(solve(problems))
    ms = (time.perf_counter() - t) * 1e3
    if ref is None:
        ref = d
    bad = sum(a != b for a, b in zip(d, ref))
    print(f"rep {k}: {ms:.1f} ms, {bad} problems differ from rep 0", flush=True)
    assert bad == 0
print("stress ok")
