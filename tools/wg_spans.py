#!/usr/bin/env python3
"""Per-workgroup start / end of the last k_score_fm launch on the global
100 MHz clock (diagnostic build: GCR_LIB=libgcr_stamps.so, `make stamps`):
how much of a launch is its tail, i.e. the spread between the workgroups of
one launch (one workgroup per CU at 4096 hypotheses).

usage: GCR_LIB=libgcr_stamps.so python tools/wg_spans.py [--workload m2|m1] [--slots 4096]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-cut-ransac_amd"))
os.environ.setdefault("GCR_LIB", "libgcr_stamps.so")

from pygcransac import _native as N  # noqa: E402
from pygcransac import synthetic as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="m2")
    ap.add_argument("--slots", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    seed = 20251121
    if a.workload == "m2":
        f0, f1, _, _, thr0, thr1 = S.problem_m2(5000, 5000, seed=seed)
        solver = N.SOLVER_SIFT22
    else:
        f0, _, thr0 = S.problem_m1(10_000, seed=seed)
        f1, thr1, solver = None, 0.0, N.SOLVER_SCALE3
    ctx = N.context(0)
    dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    f0 = np.ascontiguousarray(f0)
    f1 = None if f1 is None else np.ascontiguousarray(f1)
    ph = C.c_void_p()
    N.check(N.lib.gcr_problem_create(ctx, solver, dp(f0), f0.shape[0], dp(f1) if f1 is not None else None,
                                     0 if f1 is None else f1.shape[0], C.byref(ph)))
    p = N.default_params()
    p.scale_residual_thresh = thr0
    p.orientation_residual_thresh = thr1
    p.seed = seed
    res = (N.BatchResult * a.steps)()
    st = N.Stats()
    N.check(N.lib.gcr_problem_verify_batches(ph.value, C.byref(p), 0, a.slots, a.steps, res, C.byref(st)))
    N.check(N.lib.gcr_synchronize(ctx))
    nwg = a.slots // 16
    buf = np.zeros((4096, 3), dtype=np.uint64)
    fn = N.lib.gcr_debug_wgspans
    fn.argtypes = [C.c_void_p, C.c_size_t]
    n = fn(buf.ctypes.data, buf.nbytes)
    assert n > 0
    s = buf[:nwg].astype(np.int64)
    t0 = s[:, 0].min()
    start = (s[:, 0] - t0) * 10.0 / 1000.0          # us (100 MHz ticks)
    end = (s[:, 1] - t0) * 10.0 / 1000.0
    dur = end - start
    print(f"workgroups {nwg}: start spread {start.max():.2f} us; duration mean {dur.mean():.2f} "
          f"p50 {np.median(dur):.2f} p90 {np.percentile(dur, 90):.2f} max {dur.max():.2f} us; "
          f"launch span {end.max():.2f} us; mean/span {dur.mean() / end.max():.3f}")
    surv = s[:, 2].astype(np.float64)
    if surv.std() > 0:
        print(f"  exact-pass survivors per workgroup: mean {surv.mean():.0f} min {surv.min():.0f} max {surv.max():.0f};"
              f" correlation with duration {np.corrcoef(surv, dur)[0, 1]:.3f}")
        order = np.argsort(surv)
        q = len(order) // 4
        print(f"  duration by survivor quartile: " + ", ".join(
            f"{dur[order[k * q:(k + 1) * q]].mean():.1f}" for k in range(4)) + " us")
    hist, edges = np.histogram(dur, bins=10)
    for h, e0, e1 in zip(hist, edges[:-1], edges[1:]):
        print(f"  {e0:7.2f}-{e1:7.2f} us {h:4d} " + "#" * int(h // 2))


if __name__ == "__main__":
    main()
