"""7-point fundamental matrix (BASELINE configs[3]).

Absent from the fork (SURVEY finding 0.1) and upstream GC-RANSAC is not in the
container: parity is UNPINNED against any reference.  The oracle's FSolver
(oracle/gcr_oracle.cpp) restates the design of graph-cut-ransac_amd/csrc/fund.h
and is pinned only by synthetic two-view ground truth.  GPU <-> oracle
comparisons are bitwise: samples, attempt counts, the 1..3 models of every
sample, MSAC sums, masks, the final F and run statistics.
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

u32p = C.POINTER(C.c_uint32)


def _align(F, G):
    """F scaled by +-1 to face G (both unit Frobenius norm)."""
    return F * np.sign(np.sum(F * G))


def _sampson(F, corr):
    x1 = np.column_stack([corr[:, :2], np.ones(len(corr))])
    x2 = np.column_stack([corr[:, 2:], np.ones(len(corr))])
    Fx, Ftx = x1 @ F.T, x2 @ F
    num = np.sum(x2 * Fx, 1)
    return num * num / (Fx[:, 0] ** 2 + Fx[:, 1] ** 2 + Ftx[:, 0] ** 2 + Ftx[:, 1] ** 2)


# ------------------------------------------------------------ CPU: oracle ----
def test_oracle_recovers_ground_truth(oracle):
    corr, truth, Fgt, thr = S.problem_f(3000, 0.6, seed=4)
    r = O.find_fundamental(corr, thr, min_it=50, max_it=200000, confidence=0.99, seed=1)
    assert r["num_inliers"] > 0
    m = r["mask"]
    assert (m & truth).sum() / m.sum() > 0.97
    assert (m & truth).sum() / truth.sum() > 0.97
    F = r["H"]
    assert abs(np.linalg.norm(F) - 1.0) < 1e-12
    assert abs(np.linalg.det(F)) < 1e-9                    # rank 2
    assert np.abs(_align(F, Fgt) - Fgt).max() < 1e-2


def test_oracle_minimal_models_fit_their_sample(oracle):
    corr, _, _, _ = S.problem_f(300, 0.3, seed=2)
    counts = []
    for slot in range(64):
        inc, ms = O.f_slot(corr, 7, slot)
        if inc > 101:
            continue
        counts.append(len(ms))
        for F in ms:
            assert abs(np.linalg.norm(F) - 1.0) < 1e-12
            assert abs(np.linalg.det(F.reshape(3, 3))) < 1e-8
            # the 7 sample correspondences lie on the model exactly
            assert (O.f_residuals(corr, F) < 1e-10).sum() >= 7
    assert len(counts) > 48 and 1 <= min(counts) and max(counts) <= 3
    assert max(counts) >= 2                       # multi-model samples occur


def test_oracle_fit_reproduces_exact_geometry(oracle):
    corr, truth, Fgt, _ = S.problem_f(400, 0.0, seed=3, noise=0.0)
    F = O.f_fit(corr, np.arange(400)).reshape(3, 3)
    assert np.abs(_align(F, Fgt) - Fgt).max() < 1e-9


# ---------------------------------------------------- CPU: host fit vs oracle
def _host_fit_f(corr, idx):
    c = np.ascontiguousarray(corr, dtype=np.float64)
    i = np.ascontiguousarray(idx, dtype=np.uint32)
    out = np.zeros(9)
    rc = N.check(N.lib.gcr_host_fit_f(dp(c), c.shape[0], i.ctypes.data_as(u32p), len(i), dp(out)))
    return out if rc == 1 else None


@pytest.mark.parametrize("k", [7, 8, 49, 700, 3000])
def test_host_fit_matches_oracle_bitwise(oracle, k):
    corr, _, _, _ = S.problem_f(3500, 0.4, seed=k)
    rng = np.random.default_rng(k)
    idx = np.sort(rng.choice(len(corr), k, replace=False))
    got = _host_fit_f(corr, idx)
    exp = O.f_fit(corr, idx)
    assert (got is None) == (exp is None)
    if got is not None:
        assert np.array_equal(bits(got), bits(exp))


def test_find_fundamental_matrix_signature_and_errors():
    import inspect
    names = list(inspect.signature(pygcransac.findFundamentalMatrix).parameters)
    assert names[:13] == ["correspondences", "h1", "w1", "h2", "w2", "probabilities", "threshold", "conf",
                          "spatial_coherence_weight", "max_iters", "min_iters", "sampler", "lo_number"]
    with pytest.raises(ValueError) as e:
        pygcransac.findFundamentalMatrix(np.zeros((6, 4)), 960, 1280, 960, 1280)
    assert str(e.value) == ("Correspondences should be an array with 4 columns and at least 7 rows. "
                            "It has 4 columns and 6 rows.")
    with pytest.raises(ValueError):
        pygcransac.findFundamentalMatrix(np.zeros((10, 3)), 960, 1280, 960, 1280)


# -------------------------------------------------------------- GPU parity --
@pytest.fixture(scope="module")
def gpu():
    if N.lib.gcr_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    N.context(0)


def _finish(n0, v0, tot, thr):
    if int(n0) < 7:
        return 0, 0.0
    T = (2.25 * thr) * thr
    return int(n0), (float(tot) - float(v0)) + (float(v0) / T + float(n0))


@pytest.mark.gpu
def test_generate_matches_oracle_slots(gpu):
    corr, _, _, _ = S.problem_f(600, 0.5, seed=21)
    prob = CorrProblem(N.SOLVER_FUNDAMENTAL7, corr)
    inc, F = prob.generate(31, 4000, 384)
    multi = 0
    for s in range(384):
        oinc, oms = O.f_slot(corr, 31, 4000 + s)
        assert int(inc[s, 0]) == oinc, s
        if oinc > 101:
            assert inc[s, 1] == 255 and inc[s, 2] == 255
            continue
        k = len(oms)
        multi += k > 1
        assert [int(v) for v in inc[s, 1:]] == [0 if q < k else 255 for q in (1, 2)], s
        assert np.array_equal(bits(F[s, :k]), bits(oms)), s
    assert multi > 0


@pytest.mark.gpu
@pytest.mark.parametrize("g,widen", [(1, "1"), (2, "1"), (4, "1"), (8, "1"), (16, "1"), (32, "1"), (64, "1"), (32, "0"), (2, "0")])
def test_generate_group_widening_matches_oracle_slots(gpu, g, widen, monkeypatch):
    """k_generate_fw hands finished slots' lanes to unfinished ones; at 80 %
    outliers (7.7 attempts per slot on average, some past 64) every slot must
    still report the sequential loop's first success, for every starting
    group size, and the fixed-group kernel (GCR_GEN_WIDEN=0) the same.
    499 slots: a ragged last wave."""
    monkeypatch.setenv("GCR_GEN_G", str(g))
    monkeypatch.setenv("GCR_GEN_WIDEN", widen)
    corr, _, _, _ = S.problem_f(700, 0.8, seed=24)
    prob = CorrProblem(N.SOLVER_FUNDAMENTAL7, corr)
    inc, F = prob.generate(77, 9000, 499)
    late = 0
    for s in range(499):
        oinc, oms = O.f_slot(corr, 77, 9000 + s)
        assert int(inc[s, 0]) == oinc, (s, int(inc[s, 0]), oinc)
        late += oinc > 33
        if oinc > 101:
            assert inc[s, 1] == 255 and inc[s, 2] == 255
            continue
        k = len(oms)
        assert [int(v) for v in inc[s, 1:]] == [0 if q < k else 255 for q in (1, 2)], s
        assert np.array_equal(bits(F[s, :k]), bits(oms)), s
    assert late > 0                # some slots needed a widened second round
    # every attempt fails (all points on one line: rank-deficient 7 x 9
    # systems): every slot reports 102, written once by its group
    t = np.linspace(0.0, 500.0, 60)
    flat = np.column_stack([t, 2.0 * t + 1.0, t + 3.0, 0.5 * t])
    pf = CorrProblem(N.SOLVER_FUNDAMENTAL7, flat)
    inc, _ = pf.generate(5, 0, 131)
    for s in range(131):
        oinc, _ = O.f_slot(flat, 5, s)
        assert oinc == 102 and int(inc[s, 0]) == 102 and inc[s, 1] == 255 and inc[s, 2] == 255, s


@pytest.mark.gpu
@pytest.mark.parametrize("nh", [100, 2048, 16384, "small"])
def test_score_matches_oracle_bitwise(gpu, nh, monkeypatch):
    if nh == "small":              # launch_score_small (LO trials, refits)
        monkeypatch.setenv("GCR_DEBUG_SCORER", "small")
        nh = 200
    corr, _, _, thr = S.problem_f(1337, 0.5, seed=22)
    prob = CorrProblem(N.SOLVER_FUNDAMENTAL7, corr)
    inc, F = prob.generate(5, 0, 128)
    uniq = F[inc <= 101][:96]
    tiled = np.resize(uniq, (nh, 9))
    n0, v0, tot = prob.score(tiled, thr)
    refs = [O.f_score(corr, m, thr) for m in uniq]
    for i in range(nh):
        ref = refs[i % len(uniq)]
        cnt, val = _finish(n0[i], v0[i], tot[i], thr)
        assert cnt == (ref["count"] if ref["count"] >= 7 else 0), i
        assert bits(val) == bits(ref["value"]), i


@pytest.mark.gpu
def test_mask_matches_oracle(gpu):
    corr, _, _, thr = S.problem_f(900, 0.5, seed=23)
    prob = CorrProblem(N.SOLVER_FUNDAMENTAL7, corr)
    inc, F = prob.generate(8, 0, 32)
    for m in F[inc <= 101][:16]:
        assert np.array_equal(prob.mask(m, 0, thr), O.f_score(corr, m, thr, want_mask=True)["mask"])
        r2 = O.f_residuals(corr, m)
        t = 1.5 * thr
        assert np.array_equal(prob.mask(m, 1, thr), r2 <= t * t)


def _run_both(corr, thr, seed, **kw):
    pk = dict(min_iters=kw.get("min_it", 50), max_iters=kw.get("max_it", 10000), conf=kw.get("confidence", 0.99),
              spatial_coherence_weight=kw.get("lam", 0.0), lo_number=kw.get("lo", 50))
    r = pygcransac.findFundamentalMatrix(corr, 960, 1280, 960, 1280, threshold=thr, seed=seed, return_stats=True,
                                         batch_slots=kw.get("batch_slots", 0), **pk)
    ref = O.find_fundamental(corr, thr, min_it=pk["min_iters"], max_it=pk["max_iters"], confidence=pk["conf"],
                             lam=pk["spatial_coherence_weight"], lo=pk["lo_number"], seed=seed,
                             cell_size=P.grid_cell_sizes(corr, 960, 1280, 960, 1280, 8), cell_number=8)
    return r, ref


def _assert_same(corr, thr, seed, **kw):
    (F, mask, st), ref = _run_both(corr, thr, seed, **kw)
    rs = ref["stats"]
    assert np.array_equal(mask, ref["mask"])
    for k in ("iteration_number", "local_optimization_number", "graph_cut_number", "slots", "hypotheses"):
        assert st[k] == rs[k], k
    assert bits(st["score"]) == bits(rs["score"])
    if ref["num_inliers"] == 0:
        assert F is None
    else:
        assert np.array_equal(bits(F), bits(ref["H"]))
    return F, mask, st


@pytest.mark.gpu
@pytest.mark.parametrize("n,outl,seed", [(40, 0.2, 1), (600, 0.5, 2), (3000, 0.7, 3), (10000, 0.8, 4)])
def test_end_to_end_matches_oracle(gpu, n, outl, seed):
    corr, truth, Fgt, thr = S.problem_f(n, outl, seed=300 + seed)
    kw = dict(max_it=100000) if outl >= 0.8 else {}
    F, mask, st = _assert_same(corr, thr, seed, **kw)
    if n >= 600:
        assert (mask & truth).sum() / max(mask.sum(), 1) > 0.95
        assert np.abs(_align(F, Fgt) - Fgt).max() < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("problem_seed,seed,kw", [
    # the verdict's configs[3] case: 100 000-iteration cap, confidence 0.99
    (304, 4, dict(min_it=50, max_it=100000)),
    # bench.py's F latency call exactly: problem seed 20251121, seed 100,
    # min_iters 0, max_iters 1e7 (terminates on confidence, ~700k iterations)
    (20251121, 100, dict(min_it=0, max_it=10**7)),
])
def test_full_size_graph_cut_lo_matches_oracle(gpu, problem_seed, seed, kw):
    """configs[3] at full size with the default graph-cut LO: N = 10 000, 80 %
    outliers, spatial_coherence_weight 0.975, neighborhood_size 8 (labeling
    GCRANSAC.h:759-870 inside LO :873-1062), bitwise against the oracle's
    whole-graph BK: mask, F, iteration / LO / graph-cut counts, score."""
    corr, truth, Fgt, thr = S.problem_f(10_000, 0.8, seed=problem_seed)
    F, mask, st = _assert_same(corr, thr, seed, lam=0.975, **kw)
    assert st["graph_cut_number"] > 0
    assert (mask & truth).sum() / max(mask.sum(), 1) > 0.95


@pytest.mark.gpu
def test_spatial_weight_and_lo_budget_match_oracle(gpu):
    corr, _, _, thr = S.problem_f(800, 0.5, seed=9)
    _assert_same(corr, thr, 3, lam=0.975)
    _assert_same(corr, thr, 4, lo=0)


@pytest.mark.gpu
def test_results_independent_of_batch_size(gpu):
    corr, _, _, thr = S.problem_f(700, 0.5, seed=10)
    outs = []
    for b in (1, 37, 4096):
        (F, mask, st), _ = _run_both(corr, thr, 5, batch_slots=b, min_it=1500, max_it=1500)
        outs.append((bits(F).tolist(), mask.tolist(), st["iteration_number"], st["hypotheses"], bits(st["score"])))
    assert outs[0] == outs[1] == outs[2]


@pytest.mark.gpu
def test_degenerate_input_returns_none(gpu):
    corr = np.tile([[10.0, 10.0, 20.0, 20.0]], (50, 1))
    F, mask = pygcransac.findFundamentalMatrix(corr, 960, 1280, 960, 1280, threshold=1.0, min_iters=100,
                                               max_iters=100)
    ref = O.find_fundamental(corr, 1.0, min_it=100, max_it=100, confidence=0.99)
    assert ref["num_inliers"] == 0 and F is None and not mask.any()


@pytest.mark.gpu
def test_verify_batches_best_matches_oracle(gpu):
    corr, _, _, thr = S.problem_f(1000, 0.5, seed=12)
    prob = CorrProblem(N.SOLVER_FUNDAMENTAL7, corr)
    p = N.default_params()
    p.scale_residual_thresh = thr
    p.seed = 77
    nslots, nb = 128, 2
    out = (N.BatchResult * nb)()
    N.check(N.lib.gcr_problem_verify_batches(prob.h, C.byref(p), 0, nslots, nb, out, None))
    for b in range(nb):
        best, bslot, models, its = 0.0, -1, 0, 0
        for s in range(b * nslots, (b + 1) * nslots):
            inc, ms = O.f_slot(corr, 77, s)
            its += inc
            for m in ms:
                models += 1
                v = O.f_score(corr, m, thr)["value"]
                if best < v:
                    best, bslot = v, s
        assert out[b].models == models and out[b].iterations == its
        assert out[b].best_slot == bslot and bits(out[b].best_score) == bits(best)


@pytest.mark.gpu
def test_mixed_batch_records_match_direct_calls(gpu):
    # BASELINE configs[4] shape (mixed H / F / rectification problems), small
    from pygcransac import distributed as D

    probs = []
    for i in range(2):
        c, _, _, thr = S.problem_h(400 + 100 * i, 0.5, seed=500 + i)
        probs.append(dict(kind="homography", correspondences=c, threshold=thr, seed=i, min_iteration_number=50,
                          max_iteration_number=2000))
        c, _, _, thr = S.problem_f(600 + 100 * i, 0.5, seed=510 + i)
        probs.append(dict(kind="fundamental", correspondences=c, threshold=thr, seed=i, min_iteration_number=50,
                          max_iteration_number=5000))
    f, _, thr = S.problem_m1(400, seed=520)
    probs.append(dict(kind="scale_only", features=f, scale_residual_thresh=thr, seed=9, min_iteration_number=200,
                      max_iteration_number=2000))
    recs, local = D.solve_sharded(probs, D.gpu_solver(0))
    for i, pr in enumerate(probs):
        if pr["kind"] == "scale_only":
            continue
        fn = pygcransac.findHomography if pr["kind"] == "homography" else pygcransac.findFundamentalMatrix
        M, mask = fn(pr["correspondences"], 0, 0, 0, 0, threshold=pr["threshold"], conf=0.99,
                     max_iters=pr["max_iteration_number"], min_iters=50, seed=pr["seed"])
        assert recs[i]["num_inliers"] == int(mask.sum())
        assert np.array_equal(bits(recs[i]["H"]), bits(M))


@pytest.mark.gpu
def test_minimum_and_nonfinite_inputs_match_oracle(gpu):
    rng = np.random.default_rng(6)
    for seed in range(3):                       # exactly the minimal sample size
        c = np.column_stack([rng.uniform(0, 1000, (7, 2)), rng.uniform(0, 1000, (7, 2))])
        _assert_same(c, 1.0, seed, min_it=100, max_it=100)
    c, _, _, thr = S.problem_f(900, 0.5, seed=78)
    bad = c.copy()
    bad[::9, 3] = np.nan
    bad[::13, 0] = -np.inf
    _assert_same(bad, thr, 1)
    pure = np.column_stack([rng.uniform(0, 1280, (400, 2)), rng.uniform(0, 1280, (400, 2))])
    _assert_same(pure, 1.0, 2, min_it=500, max_it=500)
