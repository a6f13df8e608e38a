"""4-point homography estimator (BASELINE configs[2]).

This fork has no homography estimator (SURVEY finding 0.1) and upstream
GC-RANSAC is not in the container, so parity is UNPINNED against any
reference: the oracle's HSolver (oracle/gcr_oracle.cpp) is a restatement of
upstream's published structure, pinned here only by synthetic ground truth.
GPU <-> oracle comparisons are bitwise (samples, attempt counts, DLT models,
MSAC sums, masks, final H and run statistics), as for the rectification
solvers in test_gpu_parity.py.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O
import pygcransac
from pygcransac import pygcransac as P
from gcr_testutil import CorrProblem, bits, dp
from pygcransac import _native as N
from pygcransac import synthetic as S

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)


def _transfer(H, pts):
    p = np.column_stack([pts, np.ones(len(pts))]) @ H.T
    return p[:, :2] / p[:, 2:3]


# ------------------------------------------------------------ CPU: oracle ----
def test_oracle_recovers_ground_truth(oracle):
    corr, truth, Hgt, thr = S.problem_h(3000, 0.5, seed=4)
    r = O.find_homography(corr, thr, min_it=200, max_it=100000, confidence=0.99, seed=1)
    assert r["num_inliers"] > 0
    m = r["mask"]
    assert (m & truth).sum() / m.sum() > 0.97
    assert (m & truth).sum() / truth.sum() > 0.97
    grid = np.array([[x, y] for x in (0, 640, 1280) for y in (0, 480, 960)], dtype=float)
    assert np.abs(_transfer(r["H"], grid) - _transfer(Hgt, grid)).max() < 1.5
    assert r["H"][2, 2] == 1.0


def test_oracle_minimal_solver_interpolates_its_sample(oracle):
    corr, _, _, _ = S.problem_h(200, 0.3, seed=2)
    hits = 0
    for slot in range(64):
        inc, h = O.h_slot(corr, 7, slot)
        if inc > 101:
            continue
        hits += 1
        assert h[8] == 1.0
        # a DLT model from 4 points maps them exactly (up to rounding): some
        # 4 rows of the problem must have ~zero residual
        r2 = O.h_residuals(corr, h)
        assert (r2 < 1e-12).sum() >= 4
    assert hits > 48


def test_oracle_fit_reproduces_exact_homography(oracle):
    rng = np.random.default_rng(1)
    x1 = rng.uniform(0, 1000, (50, 2))
    corr = np.column_stack([x1, _transfer(S.H_GT, x1)])
    h = O.h_fit(corr, np.arange(50)).reshape(3, 3)
    assert np.allclose(h, S.H_GT / S.H_GT[2, 2], rtol=1e-9, atol=1e-12)


# ---------------------------------------------------- CPU: host fit vs oracle
def _host_fit_h(corr, idx):
    c = np.ascontiguousarray(corr, dtype=np.float64)
    i = np.ascontiguousarray(idx, dtype=np.uint32)
    out = np.zeros(9)
    rc = N.check(N.lib.gcr_host_fit_h(dp(c), c.shape[0], i.ctypes.data_as(u32p), len(i), dp(out)))
    return out if rc == 1 else None


@pytest.mark.parametrize("k", [4, 5, 28, 700, 3000])
def test_host_fit_matches_oracle_bitwise(oracle, k):
    corr, _, _, _ = S.problem_h(3500, 0.4, seed=k)
    rng = np.random.default_rng(k)
    idx = np.sort(rng.choice(len(corr), k, replace=False))
    got = _host_fit_h(corr, idx)
    exp = O.h_fit(corr, idx)
    assert (got is None) == (exp is None)
    if got is not None:
        assert np.array_equal(bits(got), bits(exp))


def test_host_fit_rejects_bad_indices():
    corr = np.zeros((10, 4))
    with pytest.raises(ValueError):
        _host_fit_h(corr, [0, 1, 2, 11])


# -------------------------------------------------------- CPU: API surface --
def test_find_homography_signature_and_errors():
    import inspect
    sig = inspect.signature(pygcransac.findHomography)
    names = list(sig.parameters)
    assert names[:13] == ["correspondences", "h1", "w1", "h2", "w2", "probabilities", "threshold", "conf",
                          "spatial_coherence_weight", "max_iters", "min_iters", "sampler", "lo_number"]
    with pytest.raises(ValueError, match=r"^Number of dimensions must be 2\.$"):
        pygcransac.findHomography(np.zeros(8), 960, 1280, 960, 1280)
    with pytest.raises(ValueError) as e:
        pygcransac.findHomography(np.zeros((3, 4)), 960, 1280, 960, 1280)
    assert str(e.value) == ("Correspondences should be an array with 4 columns and at least 4 rows. "
                            "It has 4 columns and 3 rows.")
    with pytest.raises(ValueError):
        pygcransac.findHomography(np.zeros((10, 4)), 960, 1280, 960, 1280, sampler=1)
    with pytest.raises(TypeError):
        pygcransac.findHomography(np.zeros((10, 4)), "960", 1280, 960, 1280)


# -------------------------------------------------------------- GPU parity --
def _finish(n0, v0, tot, thr):
    """MSACScoringFunction::getScore post-processing for one class, m = 4."""
    if int(n0) < 4:
        return 0, 0.0
    T = (2.25 * thr) * thr
    s = float(tot) - float(v0)
    return int(n0), s + (float(v0) / T + float(n0))


@pytest.fixture(scope="module")
def gpu():
    if N.lib.gcr_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    N.context(0)


@pytest.mark.gpu
def test_generate_matches_oracle_slots(gpu):
    corr, _, _, _ = S.problem_h(500, 0.5, seed=21)
    prob = CorrProblem(N.SOLVER_HOMOGRAPHY4, corr)
    inc, H = prob.generate(31, 4000, 512)
    for s in range(512):
        oinc, om = O.h_slot(corr, 31, 4000 + s)
        assert int(inc[s]) == oinc, s
        if oinc <= 101:
            assert np.array_equal(bits(H[s]), bits(om)), s
    assert (inc <= 101).mean() > 0.9


@pytest.mark.gpu
@pytest.mark.parametrize("g,widen", [(1, "1"), (4, "1"), (8, "1"), (16, "1"), (64, "1"), (16, "0")])
def test_generate_group_widening_matches_oracle_slots(gpu, g, widen, monkeypatch):
    """k_generate_fw<3, G> (GCR_GEN_HWIDEN=1) hands finished slots' lanes to
    unfinished ones; at 90 % outliers (9.7 attempts per slot, up to 65) every
    slot reports the sequential loop's first success, for every starting group
    size; a set where every attempt fails reports 102 everywhere.  499 slots:
    a ragged last wave."""
    monkeypatch.setenv("GCR_GEN_G", str(g))
    monkeypatch.setenv("GCR_GEN_HWIDEN", widen)
    corr, _, _, _ = S.problem_h(600, 0.9, seed=25)
    prob = CorrProblem(N.SOLVER_HOMOGRAPHY4, corr)
    inc, H = prob.generate(78, 9000, 499)
    late = 0
    for s in range(499):
        oinc, om = O.h_slot(corr, 78, 9000 + s)
        assert int(inc[s]) == oinc, (s, int(inc[s]), oinc)
        late += oinc > 16
        if oinc <= 101:
            assert np.array_equal(bits(H[s]), bits(om)), s
    assert late > 0
    t = np.linspace(0.0, 500.0, 60)
    flat = np.column_stack([t, 2.0 * t + 1.0, t + 3.0, 0.5 * t])
    inc, _ = CorrProblem(N.SOLVER_HOMOGRAPHY4, flat).generate(5, 0, 131)
    assert all(O.h_slot(flat, 5, s)[0] == 102 and int(inc[s]) == 102 for s in range(131))


@pytest.mark.gpu
@pytest.mark.parametrize("nh", [100, 2048, 16384, "small"])
def test_score_matches_oracle_bitwise(gpu, nh, monkeypatch):
    if nh == "small":              # launch_score_small (LO trials, refits)
        monkeypatch.setenv("GCR_DEBUG_SCORER", "small")
        nh = 200
    # covers the H = 4 / 16 / 64 hypotheses-per-workgroup variants
    corr, _, _, thr = S.problem_h(1337, 0.5, seed=22)
    prob = CorrProblem(N.SOLVER_HOMOGRAPHY4, corr)
    inc, H = prob.generate(5, 0, 256)
    uniq = H[inc <= 101][:96]
    tiled = np.resize(uniq, (nh, 9))
    n0, v0, tot = prob.score(tiled, thr)
    refs = [O.h_score(corr, m, thr) for m in uniq]
    for i in range(nh):
        ref = refs[i % len(uniq)]
        cnt, val = _finish(n0[i], v0[i], tot[i], thr)
        exp_cnt = ref["count"] if ref["count"] >= 4 else 0
        assert cnt == exp_cnt, i
        assert bits(val) == bits(ref["value"]), i


@pytest.mark.gpu
def test_mask_matches_oracle(gpu):
    corr, _, _, thr = S.problem_h(900, 0.5, seed=23)
    prob = CorrProblem(N.SOLVER_HOMOGRAPHY4, corr)
    inc, H = prob.generate(8, 0, 64)
    for m in H[inc <= 101][:16]:
        assert np.array_equal(prob.mask(m, 0, thr), O.h_score(corr, m, thr, want_mask=True)["mask"])
        r2 = O.h_residuals(corr, m)
        t = 1.5 * thr
        assert np.array_equal(prob.mask(m, 1, thr), r2 <= t * t)


def _run_both(corr, thr, seed, **kw):
    pk = dict(min_iters=kw.get("min_it", 50), max_iters=kw.get("max_it", 10000), conf=kw.get("confidence", 0.99),
              spatial_coherence_weight=kw.get("lam", 0.0), lo_number=kw.get("lo", 50))
    r = pygcransac.findHomography(corr, 960, 1280, 960, 1280, threshold=thr, seed=seed, return_stats=True,
                                  batch_slots=kw.get("batch_slots", 0), **pk)
    ok = dict(min_it=pk["min_iters"], max_it=pk["max_iters"], confidence=pk["conf"], lam=pk["spatial_coherence_weight"],
              lo=pk["lo_number"], seed=seed)
    # the default neighbourhood grid (8 cells per axis over the image sizes)
    ref = O.find_homography(corr, thr, cell_size=P.grid_cell_sizes(corr, 960, 1280, 960, 1280, 8), cell_number=8,
                            **ok)
    return r, ref


def _assert_same(corr, thr, seed, **kw):
    (H, mask, st), ref = _run_both(corr, thr, seed, **kw)
    rs = ref["stats"]
    assert np.array_equal(mask, ref["mask"])
    for k in ("iteration_number", "local_optimization_number", "graph_cut_number", "slots", "hypotheses"):
        assert st[k] == rs[k], k
    assert bits(st["score"]) == bits(rs["score"])
    if ref["num_inliers"] == 0:
        assert H is None
    else:
        assert np.array_equal(bits(H), bits(ref["H"]))
    return H, mask, st


@pytest.mark.gpu
@pytest.mark.parametrize("n,outl,seed", [(30, 0.3, 1), (500, 0.5, 2), (5000, 0.5, 3), (2000, 0.8, 4)])
def test_end_to_end_matches_oracle(gpu, n, outl, seed):
    corr, truth, Hgt, thr = S.problem_h(n, outl, seed=200 + seed)
    H, mask, st = _assert_same(corr, thr, seed)
    if n >= 500:
        assert (mask & truth).sum() / max(mask.sum(), 1) > 0.95


@pytest.mark.gpu
def test_spatial_weight_and_lo_budget_match_oracle(gpu):
    corr, _, _, thr = S.problem_h(800, 0.6, seed=9)
    _assert_same(corr, thr, 3, lam=0.975)
    _assert_same(corr, thr, 4, lo=0)


@pytest.mark.gpu
def test_results_independent_of_batch_size(gpu):
    corr, _, _, thr = S.problem_h(600, 0.5, seed=10)
    outs = []
    for b in (1, 37, 4096):
        (H, mask, st), _ = _run_both(corr, thr, 5, batch_slots=b, min_it=2000, max_it=2000)
        outs.append((bits(H).tolist(), mask.tolist(), st["iteration_number"], bits(st["score"])))
    assert outs[0] == outs[1] == outs[2]


@pytest.mark.gpu
def test_degenerate_input_returns_none(gpu):
    corr = np.tile([[10.0, 10.0, 20.0, 20.0]], (50, 1))      # all samples collinear / repeated
    H, mask = pygcransac.findHomography(corr, 960, 1280, 960, 1280, threshold=1.0, min_iters=100, max_iters=100)
    ref = O.find_homography(corr, 1.0, min_it=100, max_it=100, confidence=0.99)
    assert ref["num_inliers"] == 0 and H is None and not mask.any()


@pytest.mark.gpu
def test_verify_batches_best_slot_matches_oracle(gpu):
    corr, _, _, thr = S.problem_h(1000, 0.5, seed=12)
    prob = CorrProblem(N.SOLVER_HOMOGRAPHY4, corr)
    p = N.default_params()
    p.scale_residual_thresh = thr
    p.seed = 77
    nslots, nb = 256, 2
    out = (N.BatchResult * nb)()
    N.check(N.lib.gcr_problem_verify_batches(prob.h, C.byref(p), 0, nslots, nb, out, None))
    for b in range(nb):
        best, bslot, models, its = 0.0, -1, 0, 0
        for s in range(b * nslots, (b + 1) * nslots):
            inc, h = O.h_slot(corr, 77, s)
            its += inc
            if inc > 101:
                continue
            models += 1
            v = O.h_score(corr, h, thr)["value"]
            if best < v:
                best, bslot = v, s
        assert out[b].models == models and out[b].iterations == its
        assert out[b].best_slot == bslot and bits(out[b].best_score) == bits(best)


@pytest.mark.gpu
def test_minimum_and_nonfinite_inputs_match_oracle(gpu):
    rng = np.random.default_rng(5)
    for seed in range(3):                       # exactly the minimal sample size
        c = np.column_stack([rng.uniform(0, 1000, (4, 2)), rng.uniform(0, 1000, (4, 2))])
        _assert_same(c, 2.0, seed, min_it=100, max_it=100)
    c, _, _, thr = S.problem_h(600, 0.5, seed=77)
    bad = c.copy()
    bad[::9, 2] = np.nan
    bad[::13, 1] = np.inf
    _assert_same(bad, thr, 1)
    pure = np.column_stack([rng.uniform(0, 1280, (300, 2)), rng.uniform(0, 1280, (300, 2))])
    _assert_same(pure, 1.0, 2, min_it=500, max_it=500)


@pytest.mark.gpu
def test_band_prefilter_is_conservative_at_the_threshold(gpu):
    # the division-free h_band must keep every pair the exact transfer error
    # accepts: correspondences placed within a few ulps of sqrt(T) (the MSAC
    # threshold) of their model's transfer, counts and sums equal the oracle's
    rng = np.random.default_rng(1234)
    thr = 2.0
    T = (2.25 * thr) * thr
    models = []
    rows = []
    for i in range(12):
        Hm = S.H_GT * (1.0 + rng.normal(0, 1e-3, (3, 3)))
        Hm = Hm / Hm[2, 2]
        models.append(Hm.ravel())
        x1 = rng.uniform(0, 1280, (400, 2))
        w = (Hm[2, 0] * x1[:, 0] + Hm[2, 1] * x1[:, 1]) + Hm[2, 2]
        u = ((Hm[0, 0] * x1[:, 0] + Hm[0, 1] * x1[:, 1]) + Hm[0, 2]) / w
        v = ((Hm[1, 0] * x1[:, 0] + Hm[1, 1] * x1[:, 1]) + Hm[1, 2]) / w
        th = rng.uniform(0, 2 * np.pi, 400)
        rad = np.sqrt(T) * (1.0 + rng.integers(-8, 9, 400) * 2.0 ** -52) + rng.choice([0.0, 1e-9, -1e-9], 400)
        rows.append(np.column_stack([x1, u + rad * np.cos(th), v + rad * np.sin(th)]))
    corr = np.concatenate(rows)
    prob = CorrProblem(N.SOLVER_HOMOGRAPHY4, corr)
    refs = [O.h_score(corr, m, thr) for m in models]
    assert sum(r["count"] for r in refs) > 500                 # the boundary is populated
    for nh in (100, 2048, 16384):
        tiled = np.resize(np.array(models), (nh, 9))
        n0, v0, tot = prob.score(tiled, thr)
        for i in range(nh):
            ref = refs[i % len(models)]
            cnt, val = _finish(n0[i], v0[i], tot[i], thr)
            assert cnt == (ref["count"] if ref["count"] >= 4 else 0), (nh, i)
            assert bits(val) == bits(ref["value"]), (nh, i)
