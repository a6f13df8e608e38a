"""Inlier decisions in the reference's arithmetic on the GPU (csrc/exact.h).

Thresholds are placed between a pair's glibc and detmath r^2 (VERDICT round 3
probe, tests/gcr_testutil.py boundary_thresholds): the kernels flag every
decision within the proven twin-glibc bound, the engine decides them with
glibc.  The product must then equal the oracle's GLIBC mode -- the reference's
arithmetic -- in masks, counts, run statistics and model bits, and the
oracle's TWIN mode (the same decisions, twin values in the sums) bit for bit,
score included.  GCR_EXACT=0 (the twins' own decisions) must differ."""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O
from gcr_testutil import Problem, best_minimal_model, bits, boundary_thresholds, finish_score, first_member_model
from pygcransac import _native as N
from pygcransac import synthetic as S

pytestmark = pytest.mark.gpu

KW = dict(min_it=0, max_it=100_000, lo=50, seed=7, confidence=0.99)
KWB = dict(min_it=300, max_it=300, lo=0, seed=7, confidence=0.99)   # fixed budget, no LO trials
STATS = ("iteration_number", "local_optimization_number", "graph_cut_number", "slots", "hypotheses")


def _problem(kind, seed):
    if kind == N.SOLVER_SIFT22:
        fs, fo, _, _, ts, to = S.problem_m2(1500, 1500, seed=seed)
        return fs, fo, ts, to
    f, _, thr = S.problem_m1(2500, seed=seed)
    return f, None, thr, 0.0


def _oracle(kind, f0, f1, t0, t1, mode, kw=KW):
    if kind == N.SOLVER_SIFT22:
        r = O.rect_sift(f0, f1, t0, t1, math_mode=mode, **kw)
        return r, [r["scale_mask"], r["orientation_mask"]]
    r = O.rect_scale_only(f0, t0, original=kind == N.SOLVER_SCALE3_ORIGINAL, math_mode=mode, **kw)
    return r, [r["mask"]]


def _gpu(kind, f0, f1, t0, t1, kw=KW):
    import pygcransac

    pos = (0.0, kw["min_it"], kw["max_it"], kw["lo"])
    extra = dict(seed=kw["seed"], confidence=kw["confidence"], return_stats=True)
    if kind == N.SOLVER_SIFT22:
        H, sm, om, model, st = pygcransac.findRectifyingHomographySIFT(f0, f1, t0, t1, *pos, **extra)
        return H, [sm, om], model, st
    fn = (pygcransac.findRectifyingHomographyScaleOnlyOriginal if kind == N.SOLVER_SCALE3_ORIGINAL
          else pygcransac.findRectifyingHomographyScaleOnly)
    H, m, model, st = fn(f0, t0, *pos, **extra)
    return H, [m], model, st


def _model7(model, kind):
    keys = ("x0", "y0", "s", "h7", "h8", "alpha", "phi")
    return np.array([getattr(model, k) for k in (keys if kind == N.SOLVER_SIFT22 else keys[:6])])


@pytest.mark.parametrize("kind", [N.SOLVER_SCALE3, N.SOLVER_SCALE3_ORIGINAL, N.SOLVER_SIFT22])
def test_gpu_single_model_boundary_decisions(kind, monkeypatch):
    """gcr_debug_score / gcr_debug_mask at the constructed thresholds: counts
    and masks are glibc's, the raw accumulators TWIN mode's bit for bit; with
    GCR_EXACT=0 the constructed pair is decided as the twins decide it."""
    f0, f1, thr0, thr1 = _problem(kind, 5)
    r, _ = _oracle(kind, f0, f1, thr0, thr1, O.MATH_GLIBC)
    model = O.model7(r["model"])
    cases = boundary_thresholds(O, kind, f0, f1, thr0, thr1, model, per_class=10, window=1.0)
    assert len(cases) >= 4
    prob = Problem(kind, f0, f1)
    for cls, i, t0, t1 in cases:
        g = O.score(kind, f0, f1, model, t0, t1, math_mode=O.MATH_GLIBC, want_masks=True)
        p = O.score(kind, f0, f1, model, t0, t1, math_mode=O.MATH_TWIN)
        n0, n1, v0, v1, tot = prob.score_raw([model], t0, t1)
        K = 2 if f1 is not None else 1
        assert [int(n0[0]), int(n1[0])][:K] == [int(c) for c in g["counts"]][:K]
        fin = finish_score(kind, n0[0], n1[0], v0[0], v1[0], tot[0], t0, t1)
        assert bits(fin["value"]) == bits(p["value"])
        assert bits(fin["values"][:K]).tolist() == bits(p["values"][:K]).tolist()
        for c in range(2 if f1 is not None else 1):
            assert np.array_equal(prob.mask(model, c, 0, t0, t1), g["masks"][c])
        monkeypatch.setenv("GCR_EXACT", "0")
        assert prob.mask(model, cls, 0, t0, t1)[i] != g["masks"][cls][i]
        monkeypatch.delenv("GCR_EXACT")


CASES = [(N.SOLVER_SCALE3, 5), (N.SOLVER_SCALE3_ORIGINAL, 6), (N.SOLVER_SIFT22, 5), (N.SOLVER_SIFT22, 9)]


def _cases(kind, seed, anchor):
    """Boundary thresholds and the call's parameters: from the glibc run's
    final model ("final"), from the first chain member's generated model
    ("member": a decision every run takes sits at the boundary), or from the
    best generated hypothesis of a fixed-budget run without LO trials ("best":
    its MSAC lists are the refit's input)."""
    f0, f1, thr0, thr1 = _problem(kind, seed)
    kw = KWB if anchor == "best" else KW
    if anchor == "final":
        r, _ = _oracle(kind, f0, f1, thr0, thr1, O.MATH_GLIBC)
        m = O.model7(r["model"])
    elif anchor == "member":
        m = first_member_model(O, kind, f0, f1, thr0, thr1, KW["seed"])
    else:
        m = best_minimal_model(O, kind, f0, f1, thr0, thr1, KWB["seed"], KWB["max_it"])
    return (f0, f1), kw, boundary_thresholds(O, kind, f0, f1, thr0, thr1, m, per_class=4, window=1.0)


@pytest.mark.parametrize("anchor", ["final", "member", "best"])
@pytest.mark.parametrize("kind,seed", CASES)
def test_gpu_full_runs_at_boundary_thresholds(kind, seed, anchor, monkeypatch):
    """Whole pygcransac calls at the constructed thresholds: the reference's
    masks, statistics and model bits (GLIBC mode), and TWIN mode's score bits;
    the per-slot replay agrees.  With a hypothesis of the run as anchor the
    host has decided some pair with glibc."""
    (f0, f1), kw, cases = _cases(kind, seed, anchor)
    assert cases
    pairs = 0
    for cls, i, t0, t1 in cases:
        g, gm = _oracle(kind, f0, f1, t0, t1, O.MATH_GLIBC, kw)
        p, _ = _oracle(kind, f0, f1, t0, t1, O.MATH_TWIN, kw)
        H, masks, model, st = _gpu(kind, f0, f1, t0, t1, kw)
        for a, b in zip(masks, gm):
            assert np.array_equal(a, b)
        assert [st[k] for k in STATS] == [g["stats"][k] for k in STATS]
        assert np.array_equal(_model7(model, kind), O.model7(g["model"])[:len(_model7(model, kind))])
        assert bits(st["score"]) == bits(p["stats"]["score"])
        pairs += st["exact_pairs"]
        monkeypatch.setenv("GCR_REPLAY", "slots")
        H2, masks2, model2, st2 = _gpu(kind, f0, f1, t0, t1, kw)
        monkeypatch.delenv("GCR_REPLAY")
        for a, b in zip(masks2, gm):
            assert np.array_equal(a, b)
        assert np.array_equal(_model7(model2, kind), _model7(model, kind))
        assert [st2[k] for k in STATS] == [st[k] for k in STATS]
    if anchor != "final":
        assert pairs > 0                 # some decisions were taken in glibc on the host


@pytest.mark.parametrize("kind,seed", CASES)
def test_gpu_twin_decisions_differ_at_best_boundaries(kind, seed, monkeypatch):
    """GCR_EXACT=0 keeps the twins' decisions: at the best hypothesis's
    boundary thresholds most runs then differ from the reference's (which the
    default path matches, test above), and the default path flipped
    decisions on the host."""
    (f0, f1), kw, cases = _cases(kind, seed, "best")
    differ = flips = 0
    for cls, i, t0, t1 in cases:
        g, gm = _oracle(kind, f0, f1, t0, t1, O.MATH_GLIBC, kw)
        _, _, _, st = _gpu(kind, f0, f1, t0, t1, kw)
        flips += st["exact_flips"]
        monkeypatch.setenv("GCR_EXACT", "0")
        _, masks, model, st0 = _gpu(kind, f0, f1, t0, t1, kw)
        monkeypatch.delenv("GCR_EXACT")
        same = all(np.array_equal(a, b) for a, b in zip(masks, gm)) and \
            np.array_equal(_model7(model, kind), O.model7(g["model"])[:len(_model7(model, kind))])
        differ += not same
    assert flips >= 1 and 2 * differ >= len(cases)


def test_gpu_models_outside_the_bound_decided_on_the_host():
    """A scale feature outside [2^-200, 2^200] leaves exact.h's error bound
    unproven for every model (scale_unsafe): every scale decision of every
    model the replay acts on is taken on the host; still the reference's run."""
    f, _, thr = S.problem_m1(800, seed=11)
    f = f.copy()
    f[17, 2] = 1e-80                      # 2^-266: scales_in_range fails
    g, gm = _oracle(N.SOLVER_SCALE3, f, None, thr, 0.0, O.MATH_GLIBC)
    p, _ = _oracle(N.SOLVER_SCALE3, f, None, thr, 0.0, O.MATH_TWIN)
    H, masks, model, st = _gpu(N.SOLVER_SCALE3, f, None, thr, 0.0)
    assert np.array_equal(masks[0], gm[0])
    assert [st[k] for k in STATS] == [g["stats"][k] for k in STATS]
    assert np.array_equal(_model7(model, N.SOLVER_SCALE3), O.model7(g["model"])[:6])
    assert bits(st["score"]) == bits(p["stats"]["score"])
    assert st["exact_models"] > 0 and st["exact_pairs"] >= 800
