"""Device check of k_lo_chain's block-parallel exact fold (fold_exact_block,
gcr_debug_math op 7) against the sequential fp64 sum on adversarial sequences
(ties at every scale, binade crossings, zeros, subnormals, huge values, inf,
NaN, lengths around the 64-lane batch), and the small-batch scorer with the
default block fold against the one-lane fold (GCR_LO_FOLD=seq) on every
estimator."""
import ctypes as C

import numpy as np
import pytest

from fold_cases import cases, sequential
from gcr_testutil import CorrProblem, Problem
from pygcransac import _native as N
from pygcransac import synthetic as S

pytestmark = pytest.mark.gpu


def _fold(v):
    v = np.ascontiguousarray(v, dtype=np.float64)
    out = np.zeros(max(2, v.size))
    dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    N.check(N.lib.gcr_debug_math(N.context(0), 7, dp(v), None, v.size, dp(out)))
    return out[0], out[1]


def _same(a, b):
    return np.float64(a).tobytes() == np.float64(b).tobytes() or (a != a and b != b)


@pytest.mark.parametrize("name", sorted(cases()))
def test_device_fold_equals_sequential_sum(name):
    v = cases()[name]
    wide, seq = _fold(v)
    ref = sequential(v)
    assert _same(seq, ref), (seq, ref)
    assert _same(wide, ref), (wide, ref)


def test_device_fold_random():
    rng = np.random.default_rng(5)
    for _ in range(60):
        n = int(rng.integers(2, 20000))
        scale = 10.0 ** rng.uniform(-8, 8)
        v = -rng.uniform(0, scale, n)
        if rng.random() < 0.5:
            v = np.round(v / scale * 64) * scale / 64
        wide, _ = _fold(v)
        assert _same(wide, sequential(v))


def _fold3(v, h):
    v = np.ascontiguousarray(v, dtype=np.float64)
    out = np.zeros(max(7, v.size))
    hb = np.full(v.size, float(h))
    dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    N.check(N.lib.gcr_debug_math(N.context(0), 12, dp(v), dp(hb), v.size, dp(out)))
    return out[:7]


def test_device_three_chain_fold():
    """k_lo_chain's two-class fold: class 0 from +0, class 1 from +0 and
    class 1 continuing the class-0 sum, in one fold_exact_chains call."""
    rng = np.random.default_rng(12)
    named = [v for v in cases().values() if 7 <= v.size <= 8192]
    for it in range(80):
        if it < len(named):
            v = named[it]
        else:
            n = int(rng.integers(7, 8193))
            scale = 10.0 ** rng.uniform(-8, 8)
            v = -rng.uniform(0, scale, n)
            if rng.random() < 0.5:
                v = np.round(v / scale * 64) * scale / 64
        for h in {0, int(rng.integers(0, v.size + 1)), v.size // 2, v.size}:
            o = _fold3(v, h)
            r0 = sequential(v[:h])
            r1 = sequential(v[h:])
            r2 = r0
            for x in v[h:]:
                r2 = r2 + x
            for got, want in ((o[0], r0), (o[1], r1), (o[2], r2), (o[3], r0), (o[4], r1), (o[5], r2)):
                assert _same(got, want), (it, h, got, want)


def _small_scores(kind, fold, monkeypatch, split=True, nmodels=50):
    monkeypatch.setenv("GCR_DEBUG_SCORER", "small")
    if fold:
        monkeypatch.setenv("GCR_LO_FOLD", fold)
    else:
        monkeypatch.delenv("GCR_LO_FOLD", raising=False)
    monkeypatch.setenv("GCR_LO_SPLIT", "1" if split else "0")
    if kind >= N.SOLVER_HOMOGRAPHY4:
        c, _, H, thr = (S.problem_h(3000, 0.5, seed=31) if kind == N.SOLVER_HOMOGRAPHY4
                        else S.problem_f(3000, 0.6, seed=32))
        prob = CorrProblem(kind, c)
        p = N.default_params()
        p.scale_residual_thresh = thr
        rng = np.random.default_rng(3)
        k = min(nmodels, 100)
        Hs = np.ascontiguousarray(np.repeat(np.asarray(H, float).reshape(1, 9), k, 0)
                                  * (1.0 + 1e-4 * rng.standard_normal((k, 9))))
        n0 = np.zeros(k, np.uint32)
        v0 = np.zeros(k)
        tot = np.zeros(k)
        dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        N.check(N.lib.gcr_debug_score_h(prob.h, C.byref(p), dp(Hs), k, n0.ctypes.data_as(C.POINTER(C.c_uint32)),
                                        dp(v0), dp(tot)))
        return n0.tobytes() + v0.tobytes() + tot.tobytes()
    if kind == N.SOLVER_SIFT22:
        fs, fo, _, _, t0, t1 = S.problem_m2(5000, 4000, seed=33)
        prob = Problem(kind, fs, fo)
    else:
        fs, _, t0 = S.problem_m1(9000, seed=34 + kind)
        fo, t1 = None, 0.0
        prob = Problem(kind, fs, fo)
    inc, models = prob.generate(23, 0, 256)
    uniq = models[inc <= 101][:nmodels]
    return b"".join(np.asarray(a).tobytes() for a in prob.score_raw(uniq, t0, t1))


KINDS = [N.SOLVER_SCALE3, N.SOLVER_SCALE3_ORIGINAL, N.SOLVER_SIFT22, N.SOLVER_HOMOGRAPHY4, N.SOLVER_FUNDAMENTAL7]


@pytest.mark.parametrize("kind", KINDS)
def test_small_scorer_wide_fold_equals_one_lane_fold(kind, monkeypatch):
    a = _small_scores(kind, None, monkeypatch)           # default: split scorer, block fold
    b = _small_scores(kind, "seq", monkeypatch)          # k_lo_chain, one-lane folds
    c = _small_scores(kind, None, monkeypatch, split=False)   # k_lo_chain, block fold
    assert a == b
    assert a == c
    # <= kArgModels (50) rectification models travel as kernel arguments;
    # GCR_LO_ARGMODELS=0 reads them from memory instead
    for nm in (1, 50):
        d = _small_scores(kind, None, monkeypatch, nmodels=nm)
        monkeypatch.setenv("GCR_LO_ARGMODELS", "0")
        e = _small_scores(kind, None, monkeypatch, nmodels=nm)
        monkeypatch.delenv("GCR_LO_ARGMODELS")
        assert d == e


@pytest.mark.parametrize("kind", [N.SOLVER_SCALE3, N.SOLVER_SIFT22])
def test_small_scorer_many_models(kind, monkeypatch):
    # a replay chunk's worth of models (up to kSplitModels = 256) in one split launch
    a = _small_scores(kind, None, monkeypatch, nmodels=250)
    b = _small_scores(kind, "seq", monkeypatch, nmodels=250)
    c = _small_scores(kind, None, monkeypatch, split=False, nmodels=250)
    assert a == b
    assert a == c


def test_small_scorer_large_problem_keeps_per_block_folds(monkeypatch):
    # more than 2 kLoBlock pairs: the default path folds block by block one
    # value per step (the inliers no longer fit one LDS array)
    monkeypatch.setenv("GCR_DEBUG_SCORER", "small")
    fs, _, t0 = S.problem_m1(20000, seed=35)
    prob = Problem(N.SOLVER_SCALE3, fs, None)
    inc, models = prob.generate(29, 0, 128)
    uniq = models[inc <= 101][:20]
    a = b"".join(np.asarray(x).tobytes() for x in prob.score_raw(uniq, t0, 0.0))
    monkeypatch.setenv("GCR_LO_FOLD", "seq")
    b = b"".join(np.asarray(x).tobytes() for x in prob.score_raw(uniq, t0, 0.0))
    assert a == b
