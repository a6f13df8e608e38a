#!/usr/bin/env python3
"""Generate tests/golden/*.npz: seeded synthetic rectification problems and
the CPU oracle's outputs for them (SURVEY.md §8(c) golden-vector plan).

The reference itself cannot be built here (Eigen/OpenCV absent) and holds no
end-to-end fixtures, so the expected outputs are the oracle restatement's, in
both math modes:
  glibc -- the reference's own libm for every call (its arithmetic);
  twin  -- the product's arithmetic (what the GPU reproduces bitwise): every
           decision and model as glibc, the MSAC sums over detmath residuals
           (oracle/gcr_oracle.cpp, math modes).
Each file holds the inputs, the parameters and, per mode, the masks, H, the
model parameters and the run statistics.

usage: python tools/gen_golden.py [--corr-only]   (rewrites tests/golden/)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "graph-cut-ransac_amd"))

import oracle_ffi as O  # noqa: E402
from pygcransac import synthetic as S  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
SIZES = (50, 500, 2000)
PARAMS = dict(min_it=200, max_it=3000, lo=50, seed=20251121, confidence=0.95)
MODEL_KEYS = ("x0", "y0", "s", "h7", "h8", "alpha", "phi")
STAT_KEYS = ("iteration_number", "local_optimization_number", "graph_cut_number", "slots", "hypotheses")


def _pack(prefix, r, masks):
    d = {f"{prefix}_num_inliers": np.int64(r["num_inliers"]), f"{prefix}_H": r["H"],
         f"{prefix}_model": np.array([r["model"][k] for k in MODEL_KEYS]),
         f"{prefix}_stats": np.array([r["stats"][k] for k in STAT_KEYS], dtype=np.int64)}
    for name, m in masks.items():
        d[f"{prefix}_{name}"] = np.packbits(m.astype(np.uint8))
    return d


def main():
    O.build()
    os.makedirs(OUT, exist_ok=True)
    for n in SIZES:
        f, _, thr = S.problem_m1(n, seed=1000 + n)
        for original in (False, True):
            d = dict(features=f, thr=np.float64(thr), params=np.array([PARAMS[k] for k in
                                                                         ("min_it", "max_it", "lo", "seed")]))
            for mode, tag in ((O.MATH_GLIBC, "glibc"), (O.MATH_TWIN, "twin")):
                r = O.rect_scale_only(f, thr, original=original, math_mode=mode, **PARAMS)
                d.update(_pack(tag, r, {"mask": r["mask"]}))
            name = f"scale_only{'_original' if original else ''}_n{n}.npz"
            np.savez_compressed(os.path.join(OUT, name), **d)
            print(name, d["glibc_num_inliers"], d["glibc_stats"])
        fs, fo, _, _, ts, to = S.problem_m2(n, n, seed=2000 + n)
        d = dict(scale_features=fs, orientation_features=fo, thr=np.array([ts, to]),
                 params=np.array([PARAMS[k] for k in ("min_it", "max_it", "lo", "seed")]))
        for mode, tag in ((O.MATH_GLIBC, "glibc"), (O.MATH_TWIN, "twin")):
            r = O.rect_sift(fs, fo, ts, to, math_mode=mode, **PARAMS)
            d.update(_pack(tag, r, {"scale_mask": r["scale_mask"], "orientation_mask": r["orientation_mask"]}))
        name = f"sift_n{n}.npz"
        np.savez_compressed(os.path.join(OUT, name), **d)
        print(name, d["glibc_num_inliers"], d["glibc_stats"])


CORR_OUT = os.path.join(OUT, "corr")
CORR_PARAMS = dict(min_it=50, max_it=5000, lo=50, seed=20251121, confidence=0.99)


def main_corr():
    """Homography / fundamental-matrix fixtures (no reference exists: these pin
    the oracle restatement and the product against regressions)."""
    os.makedirs(CORR_OUT, exist_ok=True)
    for n in (30, 500, 2000):
        for kind, gen, fn in (("h", S.problem_h, O.find_homography), ("f", S.problem_f, O.find_fundamental)):
            c, _, _, thr = gen(max(n, 30), 0.5, seed=3000 + n)
            r = fn(c, thr, **CORR_PARAMS)
            d = dict(correspondences=c, thr=np.float64(thr),
                     params=np.array([CORR_PARAMS[k] for k in ("min_it", "max_it", "lo", "seed")]),
                     confidence=np.float64(CORR_PARAMS["confidence"]), num_inliers=np.int64(r["num_inliers"]),
                     M=r["H"], mask=np.packbits(r["mask"].astype(np.uint8)),
                     stats=np.array([r["stats"][k] for k in STAT_KEYS], dtype=np.int64))
            name = f"{kind}_n{n}.npz"
            np.savez_compressed(os.path.join(CORR_OUT, name), **d)
            print(name, d["num_inliers"], d["stats"])


if __name__ == "__main__":
    if "--corr-only" not in sys.argv:
        main()
    O.build()
    main_corr()
