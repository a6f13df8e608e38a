"""LO trials compared on approximate scores (engine.cpp score_models_approx,
kernels.hip k_lo_approx): a comparison is decided on the tree-order sums only
when the proven bound cannot change it, the round's winner is folded exactly
behind the round, and a round the bound leaves open is refolded exactly.  Runs
with the approximation off (GCR_LO_APPROX=0), on (default) and with every
round refolded (GCR_LO_APPROX=2) give the same model, masks and statistics,
and the default run matches the oracle's TWIN run."""
import numpy as np
import pytest

import oracle_ffi as O
import pygcransac
from pygcransac import synthetic as S

pytestmark = pytest.mark.gpu

_KEYS = ("iteration_number", "local_optimization_number", "graph_cut_number", "score", "lo_models", "near_ties",
         "near_tie_flips", "exact_models", "exact_pairs", "exact_flips")


def _m2(seed, n):
    fs, fo, ts, to, t0, t1 = S.problem_m2(n, n, seed=seed)
    return pygcransac.findRectifyingHomographySIFT(fs, fo, t0, t1, 0.0, 1000, 1000, 50, seed=seed, device=0,
                                                   return_stats=True)


def _m1(seed, n):
    f, _, t = S.problem_m1(n, seed=seed)
    return pygcransac.findRectifyingHomographyScaleOnly(f, t, 0.0, 1000, 1000, 50, seed=seed, device=0,
                                                        return_stats=True)


@pytest.mark.parametrize("kind,seed,n", [("m2", 3, 2000), ("m2", 11, 5000), ("m2", 109, 5000), ("m1", 7, 4000),
                                         ("m1", 21, 10000)])
def test_approx_modes_agree(monkeypatch, kind, seed, n):
    run = _m2 if kind == "m2" else _m1
    res = {}
    for mode in ("0", "1", "2", "1u"):
        monkeypatch.setenv("GCR_LO_APPROX", mode[0])
        # "1u": the approximate scores by k_lo_resid's last workgroups
        # (GCR_LO_APPROX_FUSE=1) instead of k_lo_approx's own launch
        monkeypatch.setenv("GCR_LO_APPROX_FUSE", "1" if mode == "1u" else "0")
        res[mode] = run(seed, n)
    monkeypatch.delenv("GCR_LO_APPROX")
    monkeypatch.delenv("GCR_LO_APPROX_FUSE")
    base = res["0"]
    st0 = base[-1]
    assert st0["lo_refolds"] == 0
    assert st0["local_optimization_number"] > 0
    for mode in ("1", "2", "1u"):
        r = res[mode]
        for a, b in zip(base[:-2], r[:-2]):
            assert np.array_equal(np.asarray(a), np.asarray(b)), mode
        for k in _KEYS:
            assert r[-1][k] == st0[k], (mode, k)
    # every round with trials is refolded in mode 2; the bound leaves
    # (almost) none open in mode 1
    assert res["2"][-1]["lo_refolds"] >= st0["local_optimization_number"]
    assert res["1"][-1]["lo_refolds"] <= 1
    assert res["1u"][-1]["lo_refolds"] == res["1"][-1]["lo_refolds"]


_STATS = ("iteration_number", "local_optimization_number", "graph_cut_number", "slots", "hypotheses")


def _model7(m):
    return np.array([m.x0, m.y0, m.s, m.h7, m.h8, m.alpha, m.phi])


def _assert_glibc(out, g):
    H, ms, mo, model, st = out
    assert np.array_equal(ms, g["scale_mask"]) and np.array_equal(mo, g["orientation_mask"])
    assert np.array_equal(_model7(model), O.model7(g["model"]))
    assert np.array_equal(H, g["H"])
    assert [st[k] for k in _STATS] == [g["stats"][k] for k in _STATS]


def test_approx_matches_oracle():
    fs, fo, ts, to, t0, t1 = S.problem_m2(3000, 3000, seed=17)
    out = pygcransac.findRectifyingHomographySIFT(fs, fo, t0, t1, 0.0, 1000, 1000, 50, seed=17, device=0,
                                                  return_stats=True)
    H, ms, mo, model, st = out
    # the reference's arithmetic: masks, model and homography bits, statistics
    g = O.rect_sift(fs, fo, t0, t1, min_it=1000, max_it=1000, lo=50, seed=17, math_mode=O.MATH_GLIBC)
    _assert_glibc(out, g)
    # TWIN mode: the same decisions with the product's value score, bit for bit
    tw = O.rect_sift(fs, fo, t0, t1, min_it=1000, max_it=1000, lo=50, seed=17, math_mode=O.MATH_TWIN)
    assert st["score"] == tw["stats"]["score"]
    assert st["local_optimization_number"] == tw["stats"]["local_optimization_number"]
    assert st["graph_cut_number"] == tw["stats"]["graph_cut_number"]
    assert st["near_ties"] == tw["stats"]["near_ties"]


def test_approx_at_boundary_thresholds(monkeypatch):
    """Thresholds between the glibc and twin r^2 of pairs near the threshold
    under the first chain member of the run (gcr_testutil.first_member_model:
    a decision every run with this seed takes): the approximate LO
    comparisons still give GLIBC mode's run, with some decision taken in
    glibc on the host (test_gpu_glibc.py shows such cases change the result
    when the twins decide, GCR_EXACT=0)."""
    from gcr_testutil import boundary_thresholds, first_member_model
    from pygcransac import _native as N

    fs, fo, ts, to, t0, t1 = S.problem_m2(3000, 3000, seed=17)
    m = first_member_model(O, N.SOLVER_SIFT22, fs, fo, t0, t1, 17)
    cases = boundary_thresholds(O, N.SOLVER_SIFT22, fs, fo, t0, t1, m, per_class=2, window=1.0)
    assert cases
    pairs = 0
    for cls, i, a, b in cases:
        g = O.rect_sift(fs, fo, a, b, min_it=1000, max_it=1000, lo=50, seed=17, math_mode=O.MATH_GLIBC)
        out = pygcransac.findRectifyingHomographySIFT(fs, fo, a, b, 0.0, 1000, 1000, 50, seed=17, device=0,
                                                      return_stats=True)
        _assert_glibc(out, g)
        pairs += out[-1]["exact_pairs"]
    assert pairs > 0
