"""Golden vectors of the correspondence estimators (tests/golden/corr/*.npz,
made by `tools/gen_golden.py --corr-only`): seeded homography and
fundamental-matrix problems at N = 30 / 500 / 2000 with the oracle's outputs.

There is no reference implementation of these estimators (SURVEY finding
0.1): the fixtures pin the oracle restatement and the product against
regressions, not against upstream GC-RANSAC ("parity unpinned").
CPU: the oracle reproduces every fixture exactly.  GPU: the product
reproduces every fixture bitwise, from the fixture files alone."""
import glob
import os

import numpy as np
import pytest

import oracle_ffi as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "corr")
FILES = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))
STAT_KEYS = ("iteration_number", "local_optimization_number", "graph_cut_number", "slots", "hypotheses")


def _load(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _args(d):
    min_it, max_it, lo, seed = (int(v) for v in d["params"])
    return dict(min_it=min_it, max_it=max_it, lo=lo, seed=seed, confidence=float(d["confidence"]))


def test_fixture_set_is_complete():
    names = {os.path.basename(p) for p in FILES}
    assert {f"{k}_n{n}.npz" for k in "hf" for n in (30, 500, 2000)} <= names


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(p) for p in FILES])
def test_oracle_reproduces_golden(path):
    O.build()
    d = _load(path)
    fn = O.find_homography if os.path.basename(path).startswith("h_") else O.find_fundamental
    r = fn(d["correspondences"], float(d["thr"]), **_args(d))
    n = d["correspondences"].shape[0]
    assert r["num_inliers"] == int(d["num_inliers"])
    assert np.array_equal(r["mask"], np.unpackbits(d["mask"])[:n].astype(bool))
    assert np.array_equal(r["H"].view(np.uint64), d["M"].view(np.uint64))
    assert [r["stats"][k] for k in STAT_KEYS] == d["stats"].tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(p) for p in FILES])
def test_product_reproduces_golden(path):
    import pygcransac

    d = _load(path)
    a = _args(d)
    fn = pygcransac.findHomography if os.path.basename(path).startswith("h_") else pygcransac.findFundamentalMatrix
    M, mask, st = fn(d["correspondences"], 0, 0, 0, 0, threshold=float(d["thr"]), conf=a["confidence"],
                     spatial_coherence_weight=0.0, max_iters=a["max_it"], min_iters=a["min_it"], lo_number=a["lo"],
                     seed=a["seed"], device=0, return_stats=True)
    n = d["correspondences"].shape[0]
    assert np.array_equal(mask, np.unpackbits(d["mask"])[:n].astype(bool))
    assert np.array_equal(M.view(np.uint64), d["M"].view(np.uint64))
    assert [st[k] for k in STAT_KEYS] == d["stats"].tolist()
