"""GPU <-> oracle parity (run on an MI355X: pytest -m gpu).

The oracle runs in TWIN math mode (its three hypothesis-dependent libm calls
use detmath, everything else is its own restatement), so every comparison
here is BITWISE: Philox samples, attempt counts, minimal-solver models, MSAC
counts and running sums, inlier masks, final models, H and run statistics.
The oracle's glibc mode is tied to twin mode separately (test_oracle_modes.py).
"""
import ctypes as C
import math

import numpy as np
import pytest

import oracle_ffi as O
import pygcransac
from gcr_testutil import KINDS, Problem, bits, finish_score
from pygcransac import _native as N
from pygcransac import synthetic as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    if N.lib.gcr_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    N.context(0)


def _problem_data(kind, n, seed):
    if kind == N.SOLVER_SIFT22:
        fs, fo, ts, to, thr_s, thr_o = S.problem_m2(n, n, seed=seed)
        return fs, fo, thr_s, thr_o
    f, t, thr = S.problem_m1(n, seed=seed)
    return f, None, thr, 0.0


# ----------------------------------------------------------------- math ----
def _dev_math(op, a, b=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
    out = np.zeros_like(a)
    dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    N.check(N.lib.gcr_debug_math(N.context(0), op, dp(a), dp(b) if b is not None else None, a.size, dp(out)))
    return out


def test_device_math_matches_host_bitwise():
    rng = np.random.default_rng(3)
    x = np.concatenate([np.exp(rng.uniform(-30, 30, 20000)), rng.uniform(0.5, 1.5, 20000),
                        [0.0, -0.0, -1.0, np.inf, np.nan, 5e-324, 1e-310, 1.0, 2.0]])
    got = _dev_math(0, x)
    exp = np.array([N.lib.gcr_host_log(v) for v in x])
    assert np.array_equal(bits(got), bits(exp))
    t = np.concatenate([rng.uniform(-2, 2, 20000), 10.0 ** rng.uniform(-320, 320, 2000),
                        [0.0, -0.0, np.inf, -np.inf, np.nan]])
    got = _dev_math(1, t)
    exp = np.array([N.lib.gcr_host_pow_m3(v) for v in t])
    assert np.array_equal(bits(got), bits(exp))
    y = rng.normal(size=20000) * 10.0 ** rng.uniform(-5, 5, 20000)
    xx = rng.normal(size=20000) * 10.0 ** rng.uniform(-5, 5, 20000)
    y = np.concatenate([y, [0.0, -0.0, 0.0, -0.0, 1.0, np.inf, -np.inf, np.nan]])
    xx = np.concatenate([xx, [1.0, 1.0, -1.0, -1.0, 0.0, np.inf, -np.inf, 1.0]])
    got = _dev_math(2, y, xx)
    exp = np.array([N.lib.gcr_host_atan2(a, b) for a, b in zip(y, xx)])
    assert np.array_equal(bits(got), bits(exp))
    # the value primitives (round 4): round 3's log, the model angle's sin /
    # cos, the first-octant atan of the orientation value
    for op, a, b in ((8, x, None), (9, np.concatenate([rng.uniform(-20, 20, 20000), [np.nan, np.inf, 0.0]]), None),
                     (10, np.concatenate([rng.uniform(-20, 20, 20000), [np.nan, np.inf, 0.0]]), None),
                     (11, np.abs(y[:20000]) * rng.uniform(0, 1, 20000), np.abs(y[:20000]) + 1e-300)):
        got = _dev_math(op, a, b)
        exp = np.array([N.lib.gcr_host_math(op, float(u), 0.0 if b is None else float(b[k]))
                        for k, u in enumerate(a)])
        assert np.array_equal(bits(got), bits(exp)), op


def test_clip_angle_small_equals_clip_angle():
    # the residuals clip atan2 results (|a| <= pi) and their shifts by -pi
    # with the branch-free clip_angle_small (detmath.h): same value as
    # clip_angle and the oracle's clipAngle on |a| < 4 pi and NaN
    rng = np.random.default_rng(5)
    tp = 2.0 * math.pi
    a = np.concatenate([rng.uniform(-2 * tp, 2 * tp, 100000), rng.uniform(-1e-12, 1e-12, 1000),
                        [0.0, -0.0, math.pi, -math.pi, tp, -tp, np.nextafter(tp, 0), np.nextafter(-tp, 0),
                         np.nextafter(2 * tp, 0), np.nextafter(-2 * tp, 0), -1e-300, np.nan]])
    got = _dev_math(5, a)
    assert np.array_equal(bits(got), bits(_dev_math(6, a)))
    exp = np.array([O.lib().oracle_clip_angle(v) for v in a])
    assert np.array_equal(bits(got), bits(exp))


def test_device_division_and_sqrt_are_ieee():
    rng = np.random.default_rng(4)
    a = rng.normal(size=50000) * 10.0 ** rng.uniform(-100, 100, 50000)
    b = rng.normal(size=50000) * 10.0 ** rng.uniform(-100, 100, 50000)
    assert np.array_equal(bits(_dev_math(3, a, b)), bits(a / b))
    s = np.abs(a)
    assert np.array_equal(bits(_dev_math(4, s)), bits(np.sqrt(s)))


# -------------------------------------------------------------- sampler ----
def test_sampler_matches_oracle():
    for (seed, idx, sub, stream, cls, n, m) in [(0, 0, 0, 0, 0, 10, 3), (20251121, 123456789012, 7, 0, 1, 5000, 2),
                                                 (2 ** 63 + 5, 3, 49, 1, 0, 4321, 21), (9, 1, 2, 1, 1, 15, 14)]:
        out = (C.c_uint32 * m)()
        N.check(N.lib.gcr_host_sample(seed, idx, sub, stream, cls, n, m, out))
        assert list(out) == list(O.sample(seed, idx, sub, stream, cls, n, m))


# ------------------------------------------------------- generate kernel ----
@pytest.mark.parametrize("kind", KINDS)
def test_generate_kernel_matches_oracle_slots(kind):
    f0, f1, thr0, thr1 = _problem_data(kind, 400, seed=11 + kind)
    prob = Problem(kind, f0, f1)
    seed = 977
    inc, models = prob.generate(seed, 1000, 512)
    for s in range(512):
        oinc, om = O.slot(kind, f0, f1, seed, 1000 + s)
        assert int(inc[s]) == oinc, f"slot {s}"
        if oinc <= 101:
            assert np.array_equal(bits(models[s]), bits(om)), f"slot {s}"
    assert (inc <= 101).mean() > 0.9


# ---------------------------------------------------------- score kernel ----
@pytest.mark.parametrize("kind", KINDS)
def test_score_kernel_matches_oracle_bitwise(kind):
    f0, f1, thr0, thr1 = _problem_data(kind, 1500, seed=21 + kind)
    prob = Problem(kind, f0, f1)
    inc, models = prob.generate(5, 0, 256)
    models = models[inc <= 101][:128]
    n0, n1, v0, v1, tot = prob.score_raw(models, thr0, thr1)
    for i, m in enumerate(models):
        ref = O.score(kind, f0, f1, m, thr0, thr1)
        got = finish_score(kind, n0[i], n1[i], v0[i], v1[i], tot[i], thr0, thr1)
        assert got["counts"] == [int(c) for c in ref["counts"]]
        assert np.array_equal(bits(got["values"]), bits(ref["values"]))
        assert bits(got["value"]) == bits(ref["value"])


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("nh,nf", [(1, 1337), (37, 1337), (256, 1337), (37, 5000)])
def test_small_batch_scorer_matches_oracle_bitwise(kind, nh, nf, monkeypatch):
    # launch_score_small (LO trials, refits, short replay chunks): every pair in
    # parallel, then one wave per model adds its inliers in order; ragged class
    # tails (n not a multiple of 64) exercise the padded layout, nf = 5000 two
    # 8192-value blocks of k_lo_chain (the class boundary inside the first)
    monkeypatch.setenv("GCR_DEBUG_SCORER", "small")
    f0, f1, thr0, thr1 = _problem_data(kind, nf, seed=61 + kind)
    prob = Problem(kind, f0, f1)
    inc, models = prob.generate(19, 0, 256)
    uniq = models[inc <= 101][:96]
    tiled = np.resize(uniq, (nh, 7))
    n0, n1, v0, v1, tot = prob.score_raw(tiled, thr0, thr1)
    refs = [O.score(kind, f0, f1, m, thr0, thr1) for m in uniq[:nh]]
    for i in range(nh):
        ref = refs[i % len(refs)]
        got = finish_score(kind, n0[i], n1[i], v0[i], v1[i], tot[i], thr0, thr1)
        assert got["counts"] == [int(c) for c in ref["counts"]], i
        assert np.array_equal(bits(got["values"]), bits(ref["values"])), i
        assert bits(got["value"]) == bits(ref["value"]), i


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("nh", [300, 2048, 16384])
def test_every_split_variant_matches_oracle_bitwise(kind, nh):
    # launch_score picks H = 4 / 16 / 64 hypotheses per workgroup by batch size
    # (kernels.hip split_h); tile 96 distinct models up to nh so each variant,
    # its ragged last workgroup and its round tails are exercised
    f0, f1, thr0, thr1 = _problem_data(kind, 1337, seed=91 + kind)
    prob = Problem(kind, f0, f1)
    inc, models = prob.generate(17, 0, 256)
    uniq = models[inc <= 101][:96]
    tiled = np.resize(uniq, (nh, 7))
    n0, n1, v0, v1, tot = prob.score_raw(tiled, thr0, thr1)
    refs = [O.score(kind, f0, f1, m, thr0, thr1) for m in uniq]
    for i in range(nh):
        ref = refs[i % len(uniq)]
        got = finish_score(kind, n0[i], n1[i], v0[i], v1[i], tot[i], thr0, thr1)
        assert got["counts"] == [int(c) for c in ref["counts"]], i
        assert bits(got["value"]) == bits(ref["value"]), i


@pytest.mark.parametrize("kind", KINDS)
def test_device_batch_selection_matches_host_replay(kind):
    # gcr_problem_verify_batches: k_select's first strict best per batch equals
    # the reference update rule replayed on the host over generate + score
    f0, f1, thr0, thr1 = _problem_data(kind, 900, seed=44 + kind)
    prob = Problem(kind, f0, f1)
    p = N.default_params()
    p.scale_residual_thresh, p.orientation_residual_thresh, p.seed = thr0, thr1, 123
    nslots, nb = 1500, 3
    res = (N.BatchResult * nb)()
    st = N.Stats()
    N.check(N.lib.gcr_problem_verify_batches(prob.h, C.byref(p), 7, nslots, nb, res, C.byref(st)))
    for b in range(nb):
        inc, models = prob.generate(123, 7 + b * nslots, nslots)
        ok = inc <= 101
        n0, n1, v0, v1, tot = prob.score_raw(models[ok], thr0, thr1)
        best, bj, k = 0.0, -1, 0
        for j in np.flatnonzero(ok):
            sc = finish_score(kind, n0[k], n1[k], v0[k], v1[k], tot[k], thr0, thr1)
            k += 1
            valid = kind != N.SOLVER_SIFT22 or max(abs(models[j][3]), abs(models[j][4])) < 1e-3
            if best < sc["value"] and valid:
                best, bj, cnt = sc["value"], j, sc["counts"]
        r = res[b]
        assert r.models == int(ok.sum()) and r.iterations == int(inc.astype(np.int64).sum())
        assert r.best_slot == (7 + b * nslots + bj if bj >= 0 else -1)
        if bj >= 0:
            assert bits(r.best_score) == bits(best)
            assert [r.best_inliers[0], r.best_inliers[1]] == cnt
            got = [r.best_model.x0, r.best_model.y0, r.best_model.s, r.best_model.h7, r.best_model.h8,
                   r.best_model.alpha, r.best_model.phi]
            assert np.array_equal(bits(got), bits(models[bj]))
    one = N.BatchResult()
    assert N.lib.gcr_problem_verify_batch(prob.h, C.byref(p), 7, nslots, C.byref(one), C.byref(st)) == res[0].models
    assert one.best_slot == res[0].best_slot and bits(one.best_score) == bits(res[0].best_score)


@pytest.mark.parametrize("kind", KINDS)
def test_mask_kernel_matches_oracle(kind):
    f0, f1, thr0, thr1 = _problem_data(kind, 800, seed=31 + kind)
    prob = Problem(kind, f0, f1)
    inc, models = prob.generate(8, 0, 64)
    for m in models[inc <= 101][:16]:
        ref = O.score(kind, f0, f1, m, thr0, thr1, want_masks=True)["masks"]
        assert np.array_equal(prob.mask(m, 0, 0, thr0, thr1), ref[0])
        if f1 is not None:
            assert np.array_equal(prob.mask(m, 1, 0, thr0, thr1), ref[1])
        # LO threshold rule (1.5 thr)^2 against the oracle's residuals
        r2 = O.residuals(kind, 0, f0, m)
        t = 1.5 * thr0
        assert np.array_equal(prob.mask(m, 0, 1, thr0, thr1), r2 <= t * t)


# ------------------------------------------------------------ end to end ----
def _run_product(kind, f0, f1, thr0, thr1, **kw):
    kw = dict(kw)
    kw["return_stats"] = True
    if kind == N.SOLVER_SIFT22:
        pos = {k: kw.pop(k) for k in ("spatial_coherence_weight", "min_iteration_number", "max_iteration_number",
                                      "max_local_optimization_number") if k in kw}
        r = pygcransac.findRectifyingHomographySIFT(f0, f1, thr0, thr1, **pos, **kw)
        H, ms, mo, model, st = r
        return H, (ms, mo), model, st
    fn = (pygcransac.findRectifyingHomographyScaleOnly if kind == N.SOLVER_SCALE3
          else pygcransac.findRectifyingHomographyScaleOnlyOriginal)
    r = fn(f0, thr0, **kw)
    if r[0] is None:
        return None, (r[1],), None, r[2]
    H, m, model, st = r
    return H, (m,), model, st


def _run_oracle(kind, f0, f1, thr0, thr1, seed=0, spatial_coherence_weight=0.0, min_iteration_number=10000,
                max_iteration_number=10000, max_local_optimization_number=50, confidence=0.95, **_):
    kw = dict(lam=spatial_coherence_weight, min_it=min_iteration_number, max_it=max_iteration_number,
              lo=max_local_optimization_number, confidence=confidence, seed=seed, math_mode=O.MATH_TWIN)
    if kind == N.SOLVER_SIFT22:
        r = O.rect_sift(f0, f1, thr0, thr1, **kw)
        return r, (r["scale_mask"], r["orientation_mask"])
    r = O.rect_scale_only(f0, thr0, original=(kind == N.SOLVER_SCALE3_ORIGINAL), **kw)
    return r, (r["mask"],)


def _assert_same(kind, f0, f1, thr0, thr1, **kw):
    H, masks, model, st = _run_product(kind, f0, f1, thr0, thr1, **kw)
    ref, rmasks = _run_oracle(kind, f0, f1, thr0, thr1, **kw)
    for a, b in zip(masks, rmasks):
        assert np.array_equal(a, b)
    rs = ref["stats"]
    assert st["iteration_number"] == rs["iteration_number"]
    assert st["local_optimization_number"] == rs["local_optimization_number"]
    assert st["graph_cut_number"] == rs["graph_cut_number"]
    assert st["slots"] == rs["slots"]
    assert st["hypotheses"] == rs["hypotheses"]
    assert bits(st["score"]) == bits(rs["score"])
    if ref["num_inliers"] == 0:
        assert H is None and model is None
        return st
    m = ref["model"]
    got = [model.x0, model.y0, model.s, model.h7, model.h8, model.alpha]
    exp = [m["x0"], m["y0"], m["s"], m["h7"], m["h8"], m["alpha"]]
    if kind == N.SOLVER_SIFT22:
        got.append(model.phi)
        exp.append(m["phi"])
    assert np.array_equal(bits(got), bits(exp))
    assert np.array_equal(bits(H), bits(ref["H"]))
    return st


@pytest.mark.parametrize("kind,n,seed", [
    (N.SOLVER_SCALE3, 50, 1), (N.SOLVER_SCALE3, 500, 2), (N.SOLVER_SCALE3, 2000, 3),
    (N.SOLVER_SCALE3_ORIGINAL, 500, 4), (N.SOLVER_SCALE3_ORIGINAL, 2000, 5),
    (N.SOLVER_SIFT22, 60, 6), (N.SOLVER_SIFT22, 500, 7), (N.SOLVER_SIFT22, 1500, 8),
])
def test_end_to_end_matches_oracle(kind, n, seed):
    f0, f1, thr0, thr1 = _problem_data(kind, n, seed=100 + seed)
    _assert_same(kind, f0, f1, thr0, thr1, seed=seed)


@pytest.mark.parametrize("kind", KINDS)
def test_adaptive_termination_matches_oracle(kind):
    f0, f1, thr0, thr1 = _problem_data(kind, 1000, seed=55 + kind)
    st = _assert_same(kind, f0, f1, thr0, thr1, seed=3, min_iteration_number=0, max_iteration_number=1_000_000,
                      confidence=0.99)
    assert st["iteration_number"] < 10_000


@pytest.mark.parametrize("kind", KINDS)
def test_results_independent_of_batch_size(kind):
    f0, f1, thr0, thr1 = _problem_data(kind, 600, seed=77 + kind)
    outs = []
    for b in (1, 37, 4096):
        H, masks, model, st = _run_product(kind, f0, f1, thr0, thr1, seed=9, batch_slots=b,
                                           min_iteration_number=3000, max_iteration_number=3000)
        outs.append((bits(H).tolist(), [m.tolist() for m in masks], st["iteration_number"], bits(st["score"])))
    assert outs[0] == outs[1] == outs[2]


def test_spatial_coherence_labeling_path_matches_oracle():
    f0, f1, thr0, thr1 = _problem_data(N.SOLVER_SCALE3, 700, seed=5)
    _assert_same(N.SOLVER_SCALE3, f0, f1, thr0, thr1, seed=2, spatial_coherence_weight=0.35)


@pytest.mark.parametrize("lo", [0, 1, 5])
def test_lo_trial_budget_matches_oracle(lo):
    f0, f1, thr0, thr1 = _problem_data(N.SOLVER_SIFT22, 400, seed=9)
    _assert_same(N.SOLVER_SIFT22, f0, f1, thr0, thr1, seed=4, max_local_optimization_number=lo)


# ------------------------------------------------------------- edge cases ---
def test_minimum_sizes_match_oracle():
    rng = np.random.default_rng(0)
    for seed in range(4):
        f = np.column_stack([rng.uniform(0, 100, 3), rng.uniform(0, 100, 3), rng.uniform(1, 5, 3)])
        _assert_same(N.SOLVER_SCALE3, f, None, 0.05, 0.0, seed=seed, min_iteration_number=200,
                     max_iteration_number=200)
        fs = np.column_stack([rng.uniform(0, 100, 2), rng.uniform(0, 100, 2), rng.uniform(1, 5, 2)])
        fo = np.column_stack([rng.uniform(0, 100, 2), rng.uniform(0, 100, 2), rng.uniform(0, 6, 2)])
        _assert_same(N.SOLVER_SIFT22, fs, fo, 0.05, 0.02, seed=seed, min_iteration_number=200,
                     max_iteration_number=200)


def test_pure_outliers_and_degenerate_inputs_match_oracle():
    rng = np.random.default_rng(1)
    f = np.column_stack([rng.uniform(0, 1368, 300), rng.uniform(0, 1824, 300), np.exp(rng.uniform(0, 4, 300))])
    _assert_same(N.SOLVER_SCALE3, f, None, 0.01, 0.0, seed=1, min_iteration_number=500, max_iteration_number=500)
    same = np.tile([[10.0, 20.0, 3.0]], (20, 1))          # every point identical
    _assert_same(N.SOLVER_SCALE3, same, None, 0.05, 0.0, seed=1, min_iteration_number=300,
                 max_iteration_number=300)
    line = np.column_stack([np.arange(30.0), 2 * np.arange(30.0), np.full(30, 4.0)])   # collinear
    _assert_same(N.SOLVER_SCALE3, line, None, 0.05, 0.0, seed=1, min_iteration_number=300,
                 max_iteration_number=300)
    bad = f.copy()
    bad[::7, 2] = np.nan
    bad[::11, 0] = np.inf
    _assert_same(N.SOLVER_SCALE3, bad, None, 0.05, 0.0, seed=1, min_iteration_number=500,
                 max_iteration_number=500)


def test_full_size_m1_and_m2_match_oracle_and_ground_truth():
    f, truth, thr = S.problem_m1(10_000)
    H, masks, model, st = _run_product(N.SOLVER_SCALE3, f, None, thr, 0.0, seed=0)
    gt = S.GroundTruth()
    assert abs(model.h7 - gt.h7) < 2e-6 and abs(model.h8 - gt.h8) < 2e-6 and abs(model.alpha - gt.alpha) < 1e-3
    assert (masks[0] == truth).mean() > 0.95
    _assert_same(N.SOLVER_SCALE3, f, None, thr, 0.0, seed=0)
    fs, fo, ts, to, a, b = S.problem_m2(5000, 5000)
    H, masks, model, st = _run_product(N.SOLVER_SIFT22, fs, fo, a, b, seed=0)
    assert abs(model.phi - gt.phi) < math.radians(0.5) or abs(model.phi - gt.phi - math.pi / 2) < math.radians(0.5)
    _assert_same(N.SOLVER_SIFT22, fs, fo, a, b, seed=0)


# ----------------------------------------------------- problem sharding ----
def test_gpu_solver_records_match_direct_calls():
    from pygcransac import distributed as D

    probs = []
    for i in range(3):
        fs, fo, _, _, ts, to = S.problem_m2(300 + 50 * i, 250 + 40 * i, seed=300 + i)
        probs.append(dict(kind="sift", scale_features=fs, orientation_features=fo, scale_residual_thresh=ts,
                          orientation_residual_thresh=to, max_iteration_number=2000, min_iteration_number=200,
                          seed=i))
    f, _, thr = S.problem_m1(400, seed=310)
    probs.append(dict(kind="scale_only", features=f, scale_residual_thresh=thr, seed=9,
                      min_iteration_number=200, max_iteration_number=2000))
    recs, local = D.solve_sharded(probs, D.gpu_solver(0))
    for i, pr in enumerate(probs):
        if pr["kind"] == "sift":
            H, sm, om, model = pygcransac.findRectifyingHomographySIFT(
                pr["scale_features"], pr["orientation_features"], pr["scale_residual_thresh"],
                pr["orientation_residual_thresh"], 0.0, 200, 2000, 50, seed=pr["seed"])
            n = int(sm.sum() + om.sum())
        else:
            H, m, model = pygcransac.findRectifyingHomographyScaleOnly(pr["features"], pr["scale_residual_thresh"],
                                                                       0.0, 200, 2000, 50, seed=pr["seed"])
            n = int(m.sum())
        assert recs[i]["num_inliers"] == n
        assert np.array_equal(recs[i]["H"], H)
        assert recs[i]["model"]["h7"] == model.h7 and recs[i]["model"]["h8"] == model.h8


# ------------------------------------------------------------ GPU refit ----
@pytest.mark.parametrize("ks,ko", [(40, 46), (800, 120), (2000, 260), (2500, 2500), (0, 300), (3, 1200)])
@pytest.mark.parametrize("refit", ["gram", "qr-fused", "qr-device", "qr-host"])
def test_gpu_refit_matches_host_and_oracle_bitwise(ks, ko, refit, monkeypatch):
    # the hybrid least-squares system (ns + C(no,2) rows, up to 3.1 M) solved
    # on the GPU equals the host path bit for bit.  Default ("gram", systems
    # of >= 32768 rows): the double-double Gram matrix built by one kernel
    # (gram.h), solved by pivoted Cholesky -- also equal to the oracle's
    # restatement.  GCR_REFIT=qr: the Householder QR of round 2 with its
    # driver on the device in fused passes, one pass per step, or on the host.
    # ks = 0: column 2 is all zeros (pair rows have no scale term), the
    # rank-deficient branches (nonzero = 2)
    if refit != "gram":
        monkeypatch.setenv("GCR_REFIT", "qr")
    monkeypatch.setenv("GCR_QR_DEVICE", "0" if refit == "qr-host" else "1")
    monkeypatch.setenv("GCR_QR_FUSED", "1" if refit == "qr-fused" else "0")
    fs, fo, ts, to, _, _ = S.problem_m2(5000, 5000, seed=ks + 3 * ko)
    rng = np.random.default_rng(ks + ko)
    i0 = np.sort(rng.choice(np.flatnonzero(ts), size=ks, replace=False)).astype(np.uint32)
    i1 = np.sort(rng.choice(np.flatnonzero(to), size=ko, replace=False)).astype(np.uint32)
    prob = Problem(N.SOLVER_SIFT22, fs, fo)
    u32 = C.POINTER(C.c_uint32)
    out, rcs = [], []
    for use_gpu in (1, 0):
        m = N.RectModel()
        rc = N.lib.gcr_debug_fit_nonminimal(prob.h, i0.ctypes.data_as(u32), len(i0), i1.ctypes.data_as(u32),
                                            len(i1), use_gpu, C.byref(m))
        rcs.append(rc)
        out.append(np.array([m.x0, m.y0, m.s, m.h7, m.h8, m.alpha, m.phi]))
    assert rcs[0] == rcs[1]
    if ks > 0:
        assert rcs[0] == 1
    assert np.array_equal(bits(out[0]), bits(out[1]))
    rows = ks + ko * (ko - 1) // 2
    if ko <= 300 and rcs[0] == 1 and (refit == "gram" or rows < 32768):
        exp = O.fit_nonminimal(N.SOLVER_SIFT22, fs, fo, i0, i1)
        assert np.array_equal(bits(out[0]), bits(exp))
    if rcs[0] == 1:
        # either solve within the frozen pin's tolerance of the sequential
        # Householder order
        with O.qr_order(O.QR_FROZEN):
            frz = O.fit_nonminimal(N.SOLVER_SIFT22, fs, fo, i0, i1)
        assert np.all(np.abs(out[0] - frz) <= 1e-6 * np.maximum(np.abs(frz), 1e-12))


@pytest.mark.parametrize("huge", [1e200, 1e150])
def test_gpu_gram_refit_with_overflowing_scale_rows(huge):
    # a scale inlier at huge coordinates overflows its Gram products to inf:
    # the kernel's shortcut for the pair rows (their four zero products are
    # skipped while the touched accumulators are finite) must leave the result
    # bit for bit equal to the host's full accumulation (NaN where it is NaN)
    fs, fo, ts, to, _, _ = S.problem_m2(3000, 3000, seed=77)
    rng = np.random.default_rng(78)
    i0 = np.sort(rng.choice(np.flatnonzero(ts), size=50, replace=False)).astype(np.uint32)
    i1 = np.sort(rng.choice(np.flatnonzero(to), size=400, replace=False)).astype(np.uint32)
    fs = np.array(fs, dtype=np.float64, copy=True)
    fs[i0[7], 0] = huge
    fs[i0[7], 1] = -huge
    prob = Problem(N.SOLVER_SIFT22, fs, fo)
    u32 = C.POINTER(C.c_uint32)
    out, rcs = [], []
    for use_gpu in (1, 0):
        m = N.RectModel()
        rc = N.lib.gcr_debug_fit_nonminimal(prob.h, i0.ctypes.data_as(u32), len(i0), i1.ctypes.data_as(u32),
                                            len(i1), use_gpu, C.byref(m))
        rcs.append(rc)
        out.append(np.array([m.x0, m.y0, m.s, m.h7, m.h8, m.alpha, m.phi]))
    assert rcs[0] == rcs[1]
    assert np.array_equal(bits(out[0]), bits(out[1]))


# --------------------------------------------- band prefilter, adversarial ----
def _boundary_problem(kind, rng, anchors, per=160, eps=(-1e-6, -1e-7, 0.0, 1e-7, 1e-6)):
    """Features placed at the inlier boundary (+-1.5 thr relative offsets eps)
    of each anchor model, at large coordinates; thresholds 0.05 / 1 degree."""
    thr0, thr1 = 0.05, math.radians(1.0)
    tau0, tau1 = 1.5 * thr0, 1.5 * thr1
    fs, fo = [], []
    for m in anchors:
        h7, h8, alpha, phi = m[3], m[4], m[5], m[6]
        ac = alpha ** 3
        for _ in range(per):
            x, y = rng.uniform(-5000, 5000, size=2)
            t = 1.0 - h7 * x - h8 * y
            e = eps[rng.integers(len(eps))] * rng.choice([-1, 1])
            sgn = rng.choice([-1.0, 1.0])
            if t > 0:
                k = math.exp(sgn * tau0 * (1.0 + e))
                s = t ** 3 * (ac * k if kind == N.SOLVER_SCALE3_ORIGINAL else k / ac)
            else:
                s = rng.uniform(0.5, 50)
            fs.append((x, y, s))
            if kind == N.SOLVER_SIFT22:
                rm = pygcransac.RectifyingHomography()
                rm.h7, rm.h8 = h7, h8
                u, v = rng.uniform(-3000, 3000, size=2)
                xo, yo = rm.unrectifiedPoint(u, v)
                base = phi + (math.pi / 2 if rng.random() < 0.5 else 0.0)
                th = rm.unrectifiedAngle(u, v, base + sgn * tau1 * (1.0 + e))
                fo.append((xo, yo, th))
    f0 = np.array(fs)
    f1 = np.array(fo) if fo else None
    return f0, f1, thr0, thr1


@pytest.mark.parametrize("kind", KINDS)
def test_band_prefilter_is_conservative_at_the_threshold(kind):
    # every split variant (fp32 band at H=64/16, fp64 band at H=4) must keep
    # each pair the exact residual would accept: counts and running sums equal
    # the oracle's bitwise on features placed within 1e-7 of the threshold
    rng = np.random.default_rng(1000 + kind)
    anchors = []
    for i in range(12):
        big = 2e-3 if i % 3 == 0 else 2e-4
        anchors.append(np.array([0.0, 0.0, 1.0, *rng.uniform(-big, big, size=2), rng.uniform(0.3, 3.0),
                                 rng.uniform(0, math.pi)]))
    f0, f1, thr0, thr1 = _boundary_problem(kind, rng, anchors)
    prob = Problem(kind, f0, f1)
    refs = [O.score(kind, f0, f1, m, thr0, thr1) for m in anchors]
    assert sum(r["counts"][0] for r in refs) > 100          # the boundary is populated
    for nh in (300, 2048, 16384):
        tiled = np.resize(np.array(anchors), (nh, 7))
        n0, n1, v0, v1, tot = prob.score_raw(tiled, thr0, thr1)
        for i in range(nh):
            ref = refs[i % len(anchors)]
            got = finish_score(kind, n0[i], n1[i], v0[i], v1[i], tot[i], thr0, thr1)
            assert got["counts"] == [int(c) for c in ref["counts"]], (nh, i)
            assert bits(got["value"]) == bits(ref["value"]), (nh, i)


# --------------------------------------------------- speculative prefetch ----
@pytest.mark.parametrize("kind", list(KINDS) + [N.SOLVER_HOMOGRAPHY4])
@pytest.mark.parametrize("budget", ["fixed", "adaptive"])
def test_prefetched_chunks_give_identical_runs(kind, budget, monkeypatch):
    # the next chunk generated and scored on the side stream while the host
    # replays the current one (GCR_PREFETCH) must not change anything: the
    # same slots, the same budget cut, the same replay
    if kind == N.SOLVER_HOMOGRAPHY4:
        corr, _, _, thr = S.problem_h(3000, 0.7, seed=81)
        f0, f1, thr0, thr1 = corr, None, thr, 0.0
    else:
        f0, f1, thr0, thr1 = _problem_data(kind, 2500, seed=83 + kind)
    p = N.default_params()
    p.scale_residual_thresh, p.orientation_residual_thresh, p.seed = thr0, thr1, 5
    if budget == "fixed":               # 65536-slot chunks up to a budget that cuts the last one
        p.min_iteration_number = p.max_iteration_number = 400_000 if kind in (0, 1) else 1_500_000
    else:                               # 256 -> 1024 -> 4096 ... slots, adaptive termination
        p.min_iteration_number, p.max_iteration_number, p.confidence = 0, 10**7, 0.9999999
    outs = []
    for pf in ("0", "1"):
        monkeypatch.setenv("GCR_PREFETCH", pf)
        prob = Problem(kind, f0, f1) if kind != N.SOLVER_HOMOGRAPHY4 else None
        if prob is None:
            from gcr_testutil import CorrProblem
            prob = CorrProblem(kind, f0)
        m0 = np.zeros(f0.shape[0], np.uint8)
        m1 = np.zeros(0 if f1 is None else f1.shape[0], np.uint8)
        H = np.zeros(9)
        model = N.RectModel()
        st = N.Stats()
        u8 = C.POINTER(C.c_uint8)
        n = N.check(N.lib.gcr_problem_run(prob.h, C.byref(p), m0.ctypes.data_as(u8),
                                          m1.ctypes.data_as(u8) if f1 is not None else None,
                                          H.ctypes.data_as(C.POINTER(C.c_double)), C.byref(model), C.byref(st)))
        outs.append((n, m0.tobytes(), m1.tobytes(), bits(H).tobytes(), st.iteration_number, st.hypotheses,
                     st.local_optimization_number, st.graph_cut_number, bits(st.score).tobytes(), st.slots))
        if pf == "0":
            assert st.prefetched_chunks == 0
        else:
            prefetched = st.prefetched_chunks
    assert outs[0] == outs[1]
    if budget == "fixed":
        assert prefetched > 0                                   # the path under test ran
