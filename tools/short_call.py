#!/usr/bin/env python3
"""Host-side breakdown of bench.py's timed region for a short call (the
driver's --steps 20): barrier, the verify_batches call itself (its GPU span
from the call's own event pair, stats.ms_score_kernel) and what is left.
usage: short_call.py [--steps 20] [--reps 10]"""
import argparse
import ctypes as C
import os
import statistics
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "graph-cut-ransac_amd")]
from pygcransac import _native as N  # noqa: E402
from pygcransac import synthetic as S  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--slots", type=int, default=4096)
a = ap.parse_args()
f0, f1, _, _, thr0, thr1 = S.problem_m2(5000, 5000, seed=20251121)
ctx = N.context(0)
dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
f0, f1 = np.ascontiguousarray(f0), np.ascontiguousarray(f1)
ph = C.c_void_p()
N.check(N.lib.gcr_problem_create(ctx, N.SOLVER_SIFT22, dp(f0), f0.shape[0], dp(f1), f1.shape[0], C.byref(ph)))
p = N.default_params()
p.scale_residual_thresh, p.orientation_residual_thresh, p.seed = thr0, thr1, 20251121
k = 0
for _ in range(200):                                # warm-up
    res = (N.BatchResult * a.steps)()
    N.check(N.lib.gcr_problem_verify_batches(ph.value, C.byref(p), k * a.slots, a.slots, a.steps, res, None))
    k += a.steps
rows = []
for _ in range(a.reps):
    N.check(N.lib.gcr_synchronize(ctx))
    t0 = time.perf_counter()
    res = (N.BatchResult * a.steps)()
    st = N.Stats()
    t1 = time.perf_counter()
    N.check(N.lib.gcr_problem_verify_batches(ph.value, C.byref(p), k * a.slots, a.slots, a.steps, res, C.byref(st)))
    t2 = time.perf_counter()
    N.check(N.lib.gcr_synchronize(ctx))
    t3 = time.perf_counter()
    k += a.steps
    rows.append(((t1 - t0) * 1e6, (t2 - t1) * 1e6, st.ms_score_kernel * 1e3, (t3 - t2) * 1e6, (t3 - t0) * 1e6))
for name, i in (("python setup", 0), ("verify_batches call", 1), ("its GPU span (events)", 2), ("final barrier", 3),
                ("total", 4)):
    v = [r[i] for r in rows]
    print(f"{name:24s} median {statistics.median(v):8.1f} us  min {min(v):8.1f}  max {max(v):8.1f}")
print(f"per step: {statistics.median(r[4] for r in rows) / a.steps:.2f} us")
