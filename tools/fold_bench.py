#!/usr/bin/env python3
"""Cycle counts of the small scorer's in-order folds over an LDS copy of one
value sequence (gcr_debug_math op 7): the block-parallel exact fold
(fold_exact_block, one 1024-thread workgroup) and the one-lane batched fold,
on MSAC-like sequences (-r^2 of inliers)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-cut-ransac_amd"))
from pygcransac import _native as N  # noqa: E402


def run(v):
    v = np.ascontiguousarray(v, dtype=np.float64)
    out = np.zeros(max(16, v.size))
    dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    N.check(N.lib.gcr_debug_math(N.context(0), 7, dp(v), None, v.size, dp(out)))
    return out[:6]


rng = np.random.default_rng(1)
cases = {
    "scale r^2, thr 0.05": -(rng.uniform(0, 1, 5000) * 0.05) ** 2 * 2.25,
    "orient r^2, 1 deg": -(rng.uniform(0, 1, 5000) * np.radians(1.0)) ** 2 * 2.25,
    "uniform [0, 2.25]": -rng.uniform(0, 2.25, 5000),
    "2500 values": -rng.uniform(0, 2.25, 2500),
    "8000 values": -rng.uniform(0, 2.25, 8000),
}
for name, v in cases.items():
    for _ in range(2):
        o = run(v)
    same = o[0].tobytes() == o[1].tobytes()
    print(f"{name:22s} n={v.size:5d} block {o[2]:9.0f} cyc  seq {o[3]:9.0f} cyc  ratio {o[3] / o[2]:5.2f}  "
          f"specials {o[4]:4.0f}  fallback {o[5]:1.0f}  equal {same}")


def run3(v, h):
    v = np.ascontiguousarray(v, dtype=np.float64)
    out = np.zeros(max(16, v.size))
    hb = np.full(v.size, float(h))
    dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    N.check(N.lib.gcr_debug_math(N.context(0), 12, dp(v), dp(hb), v.size, dp(out)))
    return out[:18]


# the three chains of the two-class fold (gcr_debug_math op 12: class 0 from
# +0, class 1 from +0 and from the class-0 sum) in one fold_exact_chains call
for name, v, h in (("M2-like 2 x 2500", np.concatenate([cases["scale r^2, thr 0.05"][:2500],
                                                         cases["orient r^2, 1 deg"][:2500]]), 2500),
                   ("M2-like 2 x 4000", np.concatenate([cases["scale r^2, thr 0.05"][:4000],
                                                         cases["orient r^2, 1 deg"][:4000]]), 4000),
                   ("one class 5000", cases["scale r^2, thr 0.05"], 5000)):
    for _ in range(2):
        o = run3(v, h)
    ok = all(o[i].tobytes() == o[i + 3].tobytes() for i in range(3))
    ph = np.diff(o[8:13])
    wk = np.diff(np.concatenate([o[11:12], o[13:16]]))
    print(f"3 chains {name:18s} n={v.size:5d} h={h:5d} {o[6]:9.0f} cyc  equal {ok}  phases (chunk sums, parts, "
          f"runs, walks) {' / '.join(f'{x:.0f}' for x in ph)}; wave 0: walk 0 {wk[0]:.0f}, head 2 {wk[1]:.0f}, "
          f"walk 2 {wk[2]:.0f}; walk 0 stopped at {o[16]:.0f} of {o[17]:.0f}")
