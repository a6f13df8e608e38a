"""Golden vectors (tests/golden/*.npz, made by tools/gen_golden.py): seeded
synthetic problems at N = 50 / 500 / 2000 with the oracle's outputs in the
reference's arithmetic (glibc) and in the GPU's (twin: glibc decisions and
models, detmath values in the MSAC sums -- oracle/gcr_oracle.cpp's header).
Every twin entry equals its glibc entry (regenerated in round 4 when twin mode
took its decisions from glibc; only sift_n50's model moved, to the glibc one).

CPU: the oracle still reproduces every fixture exactly (regression pin).
GPU: the product reproduces the twin outputs bitwise (masks, H, model, run
statistics) and the glibc masks exactly -- from the fixture files alone."""
import glob
import os

import numpy as np
import pytest

import oracle_ffi as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))
MODEL_KEYS = ("x0", "y0", "s", "h7", "h8", "alpha", "phi")
STAT_KEYS = ("iteration_number", "local_optimization_number", "graph_cut_number", "slots", "hypotheses")


def _load(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _masks(d, tag, names, sizes):
    return [np.unpackbits(d[f"{tag}_{nm}"])[:n].astype(bool) for nm, n in zip(names, sizes)]


def _kind(path):
    b = os.path.basename(path)
    return "sift" if b.startswith("sift") else ("original" if "original" in b else "scale")


def test_fixture_set_is_complete():
    names = {os.path.basename(p) for p in FILES}
    for n in (50, 500, 2000):
        assert {f"scale_only_n{n}.npz", f"scale_only_original_n{n}.npz", f"sift_n{n}.npz"} <= names


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(p) for p in FILES])
def test_oracle_reproduces_golden(path):
    O.build()
    d = _load(path)
    min_it, max_it, lo, seed = (int(v) for v in d["params"])
    kw = dict(min_it=min_it, max_it=max_it, lo=lo, seed=seed)
    for mode, tag in ((O.MATH_GLIBC, "glibc"), (O.MATH_TWIN, "twin")):
        if _kind(path) == "sift":
            fs, fo = d["scale_features"], d["orientation_features"]
            r = O.rect_sift(fs, fo, d["thr"][0], d["thr"][1], math_mode=mode, **kw)
            got = [r["scale_mask"], r["orientation_mask"]]
            exp = _masks(d, tag, ("scale_mask", "orientation_mask"), (len(fs), len(fo)))
        else:
            f = d["features"]
            r = O.rect_scale_only(f, float(d["thr"]), original=_kind(path) == "original", math_mode=mode, **kw)
            got, exp = [r["mask"]], _masks(d, tag, ("mask",), (len(f),))
        for a, b in zip(got, exp):
            assert np.array_equal(a, b)
        assert r["num_inliers"] == int(d[f"{tag}_num_inliers"])
        assert np.array_equal(np.array([r["model"][k] for k in MODEL_KEYS]), d[f"{tag}_model"])
        assert np.array_equal(r["H"], d[f"{tag}_H"])
        assert [r["stats"][k] for k in STAT_KEYS] == d[f"{tag}_stats"].tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(p) for p in FILES])
def test_gpu_matches_golden(path):
    import pygcransac

    d = _load(path)
    min_it, max_it, lo, seed = (int(v) for v in d["params"])
    pos = (0.0, min_it, max_it, lo)
    if _kind(path) == "sift":
        fs, fo = d["scale_features"], d["orientation_features"]
        H, sm, om, model, st = pygcransac.findRectifyingHomographySIFT(fs, fo, d["thr"][0], d["thr"][1], *pos,
                                                                       seed=seed, return_stats=True)
        got = [sm, om]
        sizes, names = (len(fs), len(fo)), ("scale_mask", "orientation_mask")
    else:
        f = d["features"]
        fn = (pygcransac.findRectifyingHomographyScaleOnlyOriginal if _kind(path) == "original"
              else pygcransac.findRectifyingHomographyScaleOnly)
        H, m, model, st = fn(f, float(d["thr"]), *pos, seed=seed, return_stats=True)
        got, sizes, names = [m], (len(f),), ("mask",)
    for a, b in zip(got, _masks(d, "twin", names, sizes)):
        assert np.array_equal(a, b)
    for a, b in zip(got, _masks(d, "glibc", names, sizes)):
        assert np.array_equal(a, b)
    assert [st[k] for k in STAT_KEYS] == d["glibc_stats"].tolist()
    exp_model = d["twin_model"]
    keys = MODEL_KEYS if _kind(path) == "sift" else MODEL_KEYS[:6]
    assert np.array_equal(np.array([getattr(model, k) for k in keys]), exp_model[:len(keys)])
    assert np.array_equal(H, d["twin_H"])
    assert [st[k] for k in STAT_KEYS] == d["twin_stats"].tolist()
    # the reference-arithmetic (glibc) model agrees within the 1e-6 contract
    g = d["glibc_model"][:len(keys)]
    assert np.all(np.abs(np.array([getattr(model, k) for k in keys]) - g) <= 1e-6 * np.maximum(np.abs(g), 1e-12))
