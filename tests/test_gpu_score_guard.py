"""The engine's score comparison on the GPU's value scores (gcr_debug_score_less:
the small scorer, then the near-tie rule of csrc/exact.h ScoreBound) takes the
reference's glibc order on ulp-perturbed neighbours whose value and glibc
orders disagree (tests/test_score_guard.py finds them with the oracle), and a
run reports the value score within the bound of the glibc score."""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O
from gcr_testutil import Problem
from pygcransac import _native as N
from test_score_guard import _disagreeing_pairs

pytestmark = pytest.mark.gpu


def _less(prob, thr0, thr1, a, b):
    p = N.default_params()
    p.scale_residual_thresh, p.orientation_residual_thresh = thr0, thr1
    ma = N.RectModel(*map(float, a))
    mb = N.RectModel(*map(float, b))
    r = N.check(N.lib.gcr_debug_score_less(prob.h, C.byref(p), C.byref(ma), C.byref(mb)))
    return bool(r & 1), bool(r & 2), bool(r & 4)


@pytest.mark.parametrize("kind,idxs", [(2, (3, 4, 5, 6)), (0, (3, 4, 5))])
def test_gpu_comparison_takes_the_glibc_order(kind, idxs):
    f0, f1, t0, t1, nb, g, v, pairs = _disagreeing_pairs(kind, 5, idxs, 10)
    prob = Problem(kind, f0, f1)
    if kind == 2:
        assert len(pairs) >= 20
    for i, j in pairs[:60]:
        d, near, vo = _less(prob, t0, t1, nb[i], nb[j])
        assert vo == (v[i] < v[j]), "GPU value scores are the oracle's TWIN scores"
        assert near and d == (g[i] < g[j]), (i, j)
    for i, j in [(0, 1), (3, 9), (len(nb) - 1, 2)]:
        d, _, _ = _less(prob, t0, t1, nb[i], nb[j])
        assert d == (g[i] < g[j])
    prob.close()


def test_run_score_within_bound_of_glibc():
    """st["score"] is the value score of the final model: it
    equals the oracle's TWIN score bit for bit, and differs from the glibc
    score by at most the proven bound; every decision of the run is glibc's
    (masks and model equal MATH_GLIBC's, test_gpu_exact.py)."""
    import pygcransac
    from pygcransac import synthetic as S
    fs, fo, _, _, ts, to = S.problem_m2(2000, 2000, seed=5)
    H, ms, mo, model, st = pygcransac.findRectifyingHomographySIFT(fs, fo, ts, to, 0.0, 1500, 1500, 50, seed=5,
                                                                   device=0, return_stats=True)
    tw = O.rect_sift(fs, fo, ts, to, min_it=1500, max_it=1500, lo=50, seed=5, math_mode=O.MATH_TWIN)
    gl = O.rect_sift(fs, fo, ts, to, min_it=1500, max_it=1500, lo=50, seed=5, math_mode=O.MATH_GLIBC)
    assert np.array_equal(ms, gl["scale_mask"]) and np.array_equal(mo, gl["orientation_mask"])
    assert st["score"] == tw["stats"]["score"]
    assert st["near_ties"] == tw["stats"]["near_ties"]
    assert abs(st["score"] - gl["stats"]["score"]) <= 1e-9 * gl["stats"]["score"]
