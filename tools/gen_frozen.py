#!/usr/bin/env python3
"""Generate tests/golden/frozen/*.npz: the oracle's outputs with its
least-squares fits in the FROZEN sequential reduction order
(oracle_set_qr_order(1), round 0's `s += f(i)` in row order).

The regular golden fixtures (tools/gen_golden.py) follow the engine's blocked
reduction order, so the product agrees with them bitwise -- but that order is
the product's choice (Eigen's own order is unpinned, no Eigen here), and each
change of it has so far redefined the oracle and the fixtures with it.  These
files never change: tests hold every product result to them with a tolerance
(masks identical, models within 1e-6 relative), so a later change of the
product's reduction order is measured against a fixed point instead.

Per problem: the regular fixture it belongs to (or the seeded generator call
and a SHA-256 of the features it must produce), the call parameters, and per
math mode the masks, H, model and run statistics.

usage: python tools/gen_frozen.py      (writes tests/golden/frozen/; run once)
"""
import glob
import hashlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "graph-cut-ransac_amd"))

import oracle_ffi as O  # noqa: E402
from pygcransac import synthetic as S  # noqa: E402
from pygcransac import pygcransac as P  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")
OUT = os.path.join(GOLDEN, "frozen")
MODEL_KEYS = ("x0", "y0", "s", "h7", "h8", "alpha", "phi")
STAT_KEYS = ("iteration_number", "local_optimization_number", "graph_cut_number", "slots", "hypotheses")
# full-size problems: the bench's own workloads (bench.py workload_problem,
# problem seed 20251121) at its 0.99-confidence latency call (seeds 100, 101)
FULL_CALL = dict(min_it=0, max_it=10**7, lo=50, confidence=0.99)
FULL_SEEDS = (100, 101)


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()


def pack(prefix, r, masks):
    d = {f"{prefix}_num_inliers": np.int64(r["num_inliers"]), f"{prefix}_H": np.asarray(r["H"]),
         f"{prefix}_stats": np.array([r["stats"][k] for k in STAT_KEYS], dtype=np.int64)}
    if "model" in r:
        d[f"{prefix}_model"] = np.array([r["model"][k] for k in MODEL_KEYS])
    for name, m in masks.items():
        d[f"{prefix}_{name}"] = np.packbits(m.astype(np.uint8))
    return d


def rect(kind, f0, f1, thr, kw):
    out = {}
    for mode, tag in ((O.MATH_GLIBC, "glibc"), (O.MATH_TWIN, "twin")):
        if kind == "sift":
            r = O.rect_sift(f0, f1, thr[0], thr[1], math_mode=mode, **kw)
            out.update(pack(tag, r, {"scale_mask": r["scale_mask"], "orientation_mask": r["orientation_mask"]}))
        else:
            r = O.rect_scale_only(f0, float(thr), original=kind == "original", math_mode=mode, **kw)
            out.update(pack(tag, r, {"mask": r["mask"]}))
    return out


def main():
    O.build()
    os.makedirs(OUT, exist_ok=True)
    with O.qr_order(O.QR_FROZEN):
        for path in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
            with np.load(path, allow_pickle=False) as z:
                d = {k: z[k] for k in z.files}
            b = os.path.basename(path)
            kind = "sift" if b.startswith("sift") else ("original" if "original" in b else "scale")
            min_it, max_it, lo, seed = (int(v) for v in d["params"])
            kw = dict(min_it=min_it, max_it=max_it, lo=lo, seed=seed)
            if kind == "sift":
                res = rect(kind, d["scale_features"], d["orientation_features"], d["thr"], kw)
            else:
                res = rect(kind, d["features"], None, d["thr"], kw)
            np.savez_compressed(os.path.join(OUT, b), source=np.str_(b), **res)
            print(b, res["glibc_num_inliers"], res["glibc_stats"])
        for path in sorted(glob.glob(os.path.join(GOLDEN, "corr", "*.npz"))):
            with np.load(path, allow_pickle=False) as z:
                d = {k: z[k] for k in z.files}
            b = os.path.basename(path)
            min_it, max_it, lo, seed = (int(v) for v in d["params"])
            fn = O.find_homography if b.startswith("h_") else O.find_fundamental
            r = fn(d["correspondences"], float(d["thr"]), min_it=min_it, max_it=max_it, lo=lo, seed=seed,
                   confidence=float(d["confidence"]))
            np.savez_compressed(os.path.join(OUT, "corr_" + b), source=np.str_("corr/" + b),
                                **pack("twin", r, {"mask": r["mask"]}))
            print("corr_" + b, r["num_inliers"], r["stats"])
        # full size: M2 (the headline workload) and F with graph-cut LO (configs[3])
        fs, fo, _, _, ts, to = S.problem_m2(5000, 5000, seed=20251121)
        for s in FULL_SEEDS:
            kw = dict(FULL_CALL, seed=s)
            res = rect("sift", fs, fo, (ts, to), kw)
            name = f"full_m2_seed{s}.npz"
            np.savez_compressed(os.path.join(OUT, name), generator=np.str_("problem_m2(5000, 5000, seed=20251121)"),
                                features_sha256=np.str_(sha(fs, fo)), thr=np.array([ts, to]),
                                params=np.array([kw["min_it"], kw["max_it"], kw["lo"], s]),
                                confidence=np.float64(kw["confidence"]), **res)
            print(name, res["glibc_num_inliers"], res["glibc_stats"])
        c, _, _, thr = S.problem_f(10_000, 0.8, seed=20251121)
        cells = P.grid_cell_sizes(c, 960, 1280, 960, 1280, 8)
        s = FULL_SEEDS[0]
        r = O.find_fundamental(c, thr, min_it=0, max_it=10**7, lo=50, confidence=0.99, lam=0.975, seed=s,
                               cell_size=cells, cell_number=8)
        name = f"full_f_lam0975_seed{s}.npz"
        np.savez_compressed(os.path.join(OUT, name), generator=np.str_("problem_f(10000, 0.8, seed=20251121)"),
                            features_sha256=np.str_(sha(c)), thr=np.float64(thr),
                            params=np.array([0, 10**7, 50, s]), confidence=np.float64(0.99), lam=np.float64(0.975),
                            **pack("twin", r, {"mask": r["mask"]}))
        print(name, r["num_inliers"], r["stats"])


if __name__ == "__main__":
    main()
