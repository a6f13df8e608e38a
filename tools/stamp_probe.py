#!/usr/bin/env python3
"""Where a k_score_fm launch spends its cycles (diagnostic build only).

Loads libgcr_stamps.so (``make -C graph-cut-ransac_amd/csrc stamps``), runs
verify batches of the bench workload, and prints the s_memtime segment shares
of the last launch for the first workgroups: compute waves (band, wait for the
chain, exact pass, pad + publish) and the chain wave (waiting for runs vs
folding them).  The stamps' own fences slow the kernel: read the shares, not
the absolute length.

usage: GCR_LIB=libgcr_stamps.so python tools/stamp_probe.py [--workload m2|m1|h] [--slots 4096]
"""
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

WG, WAVES, ROUNDS, SLOTS = 4, 16, 16, 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="m2")
    ap.add_argument("--slots", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=20)
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
    buf = np.zeros((WG, WAVES, ROUNDS, SLOTS), dtype=np.uint64)
    fn = N.lib.gcr_debug_stamps
    fn.argtypes = [C.c_void_p, C.c_size_t]
    fn.restype = C.c_int
    if fn(buf.ctypes.data, buf.nbytes) < 0:
        raise SystemExit("gcr_debug_stamps failed")
    b = buf.astype(np.int64)
    for wg in range(WG):
        t0 = b[wg, 0, 15, 5]
        print(f"== workgroup {wg}: gen {b[wg, 0, 15, 6] - t0} cyc, setup {b[wg, 0, 15, 7] - b[wg, 0, 15, 6]} cyc")
        rounds = [r for r in range(ROUNDS - 1) if b[wg, 0, r, 0] != 0]
        tot = {"band": 0, "wait": 0, "exact": 0, "pad": 0}
        for r in rounds:
            row = []
            for w in range(15):
                s = b[wg, w, r]
                seg = dict(band=s[1] - s[0], wait=s[2] - s[1], exact=s[3] - s[2], pad=s[4] - s[3])
                for k in tot:
                    tot[k] += seg[k]
                row.append(f"{seg['band']:5d}/{seg['wait']:5d}/{seg['exact']:5d}/{int(s[6]):4d}")
            c = b[wg, 15, r]
            print(f"r{r:2d} start(w0)={b[wg, 0, r, 0] - t0:7d} chain start={c[0] - t0:7d} end={c[4] - t0:7d} "
                  f"wait={c[1]:6d} fold={c[2]:6d} | w0 {row[0]} w7 {row[7]} w14 {row[14]}")
        n = max(1, 15 * len(rounds))
        end = max(b[wg, w, rounds[-1], 4] for w in range(16)) - t0 if rounds else 0
        print(f"   mean per wave-round: " + ", ".join(f"{k} {v / n:.0f}" for k, v in tot.items())
              + f"  | kernel span {end} cyc")


if __name__ == "__main__":
    main()
