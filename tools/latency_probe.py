#!/usr/bin/env python3
"""Wall time to 0.99 confidence, broken down: the full Python call, the C ABI
call alone, and the engine's own phase timers.  M2 workload (bench.py's).

usage: python tools/latency_probe.py [--reps 10]"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-cut-ransac_amd"))

import numpy as np  # noqa: E402

import pygcransac  # noqa: E402
from pygcransac import _native as N  # noqa: E402
from pygcransac import synthetic as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    fs, fo, _, _, ts, to = S.problem_m2(5000, 5000, seed=20251121)
    ctx = N.context(0)
    rows = []
    for r in range(a.reps):
        t0 = time.perf_counter()
        out = pygcransac.findRectifyingHomographySIFT(fs, fo, ts, to, 0.0, 0, 10**7, 50, seed=100 + r,
                                                      confidence=0.99, return_stats=True)
        t_py = (time.perf_counter() - t0) * 1e3
        p = N.default_params()
        p.scale_residual_thresh, p.orientation_residual_thresh = ts, to
        p.min_iteration_number, p.max_iteration_number, p.confidence, p.seed = 0, 10**7, 0.99, 100 + r
        ms_, mo_ = np.zeros(len(fs), np.uint8), np.zeros(len(fo), np.uint8)
        H, m, st = np.zeros(9), N.RectModel(), N.Stats()
        dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        u8 = lambda x: x.ctypes.data_as(C.POINTER(C.c_uint8))  # noqa: E731
        fsc, foc = np.ascontiguousarray(fs), np.ascontiguousarray(fo)
        t0 = time.perf_counter()
        N.lib.gcr_rect_sift(ctx, dp(fsc), len(fs), dp(foc), len(fo), C.byref(p), u8(ms_), u8(mo_), dp(H),
                            C.byref(m), C.byref(st))
        t_abi = (time.perf_counter() - t0) * 1e3
        s = out[-1]
        rows.append(dict(py_ms=t_py, abi_ms=t_abi, **{k: s[k] for k in (
            "ms_setup", "ms_generate", "ms_score", "ms_replay", "ms_lo", "ms_lo_lists", "ms_lo_fit", "ms_lo_score",
            "ms_refit", "ms_total",
            "iteration_number", "graph_cut_number", "lo_models", "launches")}))
    for row in rows:
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in row.items()}))
    med = {k: float(np.median([r[k] for r in rows[1:]])) for k in rows[0]}
    print("median(excl. first):", json.dumps({k: round(v, 3) for k, v in med.items()}))


if __name__ == "__main__":
    main()
