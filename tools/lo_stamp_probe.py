#!/usr/bin/env python3
"""Where one small-batch scoring launch (k_lo_chain) spends its cycles
(diagnostic build libgcr_stamps.so only; make -C graph-cut-ransac_amd/csrc
stamps).  Scores the LO-like M2 models (the generated hypotheses with the
most inliers) through gcr_debug_score with GCR_DEBUG_SCORER=small and prints,
for the first workgroups, the s_memtime segments: prologue, per pair block
(residuals + ballots, chunk prefix, compaction) per wave, and the final folds.

usage: python tools/lo_stamp_probe.py [--models 1]"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-cut-ransac_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ.setdefault("GCR_LIB", "libgcr_stamps.so")
os.environ["GCR_DEBUG_SCORER"] = "small"
os.environ["GCR_LO_SPLIT"] = "0"                    # k_lo_chain (the split scorer has no stamps)

import ctypes as C  # noqa: E402

from gcr_testutil import Problem  # noqa: E402
from pygcransac import _native as N  # noqa: E402
from pygcransac import synthetic as S  # noqa: E402

WG, WAVES, ROUNDS, SLOTS = 4, 16, 16, 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", type=int, default=1)
    a = ap.parse_args()
    fs, fo, _, _, t0, t1 = S.problem_m2(5000, 5000, seed=20251121)
    prob = Problem(N.SOLVER_SIFT22, fs, fo)
    inc, models = prob.generate(7, 0, 4096)
    live = models[inc <= 101]
    n0, n1, _, _, _ = prob.score_raw(live, t0, t1)
    order = sorted(range(len(live)), key=lambda i: -(int(n0[i]) + int(n1[i])))
    ms = live[order[:a.models]]
    for _ in range(3):
        prob.score_raw(ms, t0, t1)
    buf = np.zeros((WG, WAVES, ROUNDS, SLOTS), dtype=np.uint64)
    fn = N.lib.gcr_debug_stamps
    fn.argtypes = [C.c_void_p, C.c_size_t]
    fn.restype = C.c_int
    if fn(buf.ctypes.data, buf.nbytes) < 0:
        raise SystemExit("gcr_debug_stamps failed")
    b = buf.astype(np.int64)
    for wg in range(min(WG, a.models)):
        t0_ = b[wg, 0, 14, 0]
        print(f"== workgroup {wg}: prologue {b[wg, 0, 14, 1] - t0_} cyc")
        for blk in range(2):
            if b[wg, 0, blk, 0] == 0:
                continue
            res = [b[wg, w, blk, 0] - t0_ for w in range(16)]
            print(f"  block {blk}: residuals done (w0 / min / max over waves) {res[0]} / {min(res)} / {max(res)}, "
                  f"prefix done {b[wg, 0, blk, 1] - t0_}, compaction done {b[wg, 0, blk, 2] - t0_}")
        s = b[wg, 0, 14]
        print(f"  folds (all chains, one fold_exact_chains call): start {s[2] - t0_}, {s[3] - s[2]} cyc;"
              f" end {s[3] - t0_} cyc")


if __name__ == "__main__":
    main()
