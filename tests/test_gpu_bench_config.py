"""Parity of the EXACT kernels behind bench.py's numbers, at the bench's own
configurations (run on an MI355X: pytest -m gpu).

bench.py's step is gcr_problem_verify_batches: at 4096 slots per launch the
fused generate + score + per-workgroup-best kernel k_score_fm<K, 16, true>
plus k_select_wg, consecutive launches chained (each launch's look-ahead wave
generates the next batch's slots, which NB >= 2 exercises); at 16384 slots k_score_split<K, 64, 120, true>; the
homography generates in k_generate<3, 16> and scores in k_score_fm<3, 16,
false>; the fundamental matrix at 14848 slots (bench F_SLOTS; 3712 before
round 5) in k_generate_fw + k_compact + k_score_fm<4, 16, false> (f_band prefilter,
compaction map).  Correspondence batches run as a two-stream pipeline (batch
b + 1 generated on the side stream while batch b is scored, alternating
buffer sets), which the NB consecutive batches exercise.  Each batch's
record is checked against a pure ORACLE replay of the same slots: the
oracle's Philox sampler and minimal solvers (O.slot / h_slot / f_slot), its
twin-math MSAC score of every model, and the reference's update rule
`best < score && isValidModel` in slot order (GCRANSAC.h:440-446,
MSAC_scoring_function.hpp:108-127).  Full-size problems (M2 5000 + 5000, M1
10 000, H 5000, F 10 000 at 80 % outliers), the bench's seed, three
consecutive batches from an unaligned slot.
"""
import ctypes as C
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle_ffi as O
from gcr_testutil import CorrProblem, Problem, bits
from pygcransac import _native as N
from pygcransac import synthetic as S

pytestmark = pytest.mark.gpu

SEED = 20251121          # bench.py's problem and sampler seed (rank 0)
NB = 3
SLOT0 = 7
THREADS = 16             # the box's CPU share; ctypes releases the GIL in the oracle


@pytest.fixture(scope="module", autouse=True)
def _device():
    if N.lib.gcr_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    N.context(0)
    O.lib()


def _pmap(fn, items):
    with ThreadPoolExecutor(THREADS) as ex:
        return list(ex.map(fn, items, chunksize=64))


def _verify(h, thr0, thr1, nslots):
    p = N.default_params()
    p.scale_residual_thresh, p.orientation_residual_thresh, p.seed = thr0, thr1, SEED
    res = (N.BatchResult * NB)()
    st = N.Stats()
    N.check(N.lib.gcr_problem_verify_batches(h, C.byref(p), SLOT0, nslots, NB, res, C.byref(st)))
    return res


def _rect_oracle_slot(args):
    kind, f0, f1, thr0, thr1, s = args
    inc, m = O.slot(kind, f0, f1, SEED, s)
    if inc > 101:
        return inc, None, None
    sc = O.score(kind, f0, f1, m, thr0, thr1)
    return inc, m, sc


def _rect_problem(kind):
    if kind == N.SOLVER_SIFT22:
        fs, fo, _, _, ts, to = S.problem_m2(5000, 5000, seed=SEED)
        return fs, fo, ts, to
    f, _, thr = S.problem_m1(10_000, seed=SEED)
    return f, None, thr, 0.0


@pytest.mark.parametrize("nslots", [4096, 16384])
@pytest.mark.parametrize("kind", [N.SOLVER_SIFT22, N.SOLVER_SCALE3])
def test_fused_verify_kernel_matches_oracle_replay_at_bench_config(kind, nslots):
    f0, f1, thr0, thr1 = _rect_problem(kind)
    prob = Problem(kind, f0, f1)
    res = _verify(prob.h, thr0, thr1, nslots)
    for b in range(NB):
        s0 = SLOT0 + b * nslots
        outs = _pmap(_rect_oracle_slot, [(kind, prob.f0, prob.f1, thr0, thr1, s) for s in range(s0, s0 + nslots)])
        models = iters = 0
        best, bslot, bcnt, bmodel = 0.0, -1, None, None
        for j, (inc, m, sc) in enumerate(outs):
            iters += inc
            if m is None:
                continue
            models += 1
            valid = kind != N.SOLVER_SIFT22 or max(abs(m[3]), abs(m[4])) < 1e-3     # two_sift.hpp:45-61
            if best < sc["value"] and valid:
                best, bslot, bcnt, bmodel = sc["value"], s0 + j, [int(c) for c in sc["counts"]], m
        r = res[b]
        assert r.models == models, (b, r.models, models)
        assert r.iterations == iters, b
        assert r.best_slot == bslot, (b, r.best_slot, bslot)
        assert bslot >= 0                        # 50 % outliers: every batch finds a model
        assert bits(r.best_score) == bits(best), b
        cnt = [r.best_inliers[0], r.best_inliers[1]]
        assert cnt == bcnt, (b, cnt, bcnt)
        got = [r.best_model.x0, r.best_model.y0, r.best_model.s, r.best_model.h7, r.best_model.h8,
               r.best_model.alpha, r.best_model.phi]
        assert np.array_equal(bits(got), bits(bmodel)), b


def _h_oracle_slot(args):
    corr, thr, s = args
    inc, h = O.h_slot(corr, SEED, s)
    if inc > 101:
        return inc, []
    return inc, [O.h_score(corr, h, thr)]


def _f_oracle_slot(args):
    corr, thr, s = args
    inc, ms = O.f_slot(corr, SEED, s)
    return inc, [O.f_score(corr, m, thr) for m in ms]


@pytest.mark.parametrize("solver,nslots", [(N.SOLVER_HOMOGRAPHY4, 4096), (N.SOLVER_FUNDAMENTAL7, 3712),
                                           (N.SOLVER_FUNDAMENTAL7, 14848)])
def test_correspondence_verify_matches_oracle_replay_at_bench_config(solver, nslots):
    if solver == N.SOLVER_HOMOGRAPHY4:
        corr, _, _, thr = S.problem_h(5000, 0.5, seed=SEED)
        fn = _h_oracle_slot
    else:
        corr, _, _, thr = S.problem_f(10_000, 0.8, seed=SEED)
        fn = _f_oracle_slot
    prob = CorrProblem(solver, corr)
    res = _verify(prob.h, thr, 0.0, nslots)
    for b in range(NB):
        s0 = SLOT0 + b * nslots
        outs = _pmap(fn, [(prob.c, thr, s) for s in range(s0, s0 + nslots)])
        models = iters = 0
        best, bslot, bcnt = 0.0, -1, None
        for j, (inc, scores) in enumerate(outs):
            iters += inc
            for sc in scores:
                models += 1
                if best < sc["value"]:
                    best, bslot, bcnt = sc["value"], s0 + j, sc["count"]
        r = res[b]
        assert r.models == models and r.iterations == iters, b
        assert r.best_slot == bslot and bslot >= 0, (b, r.best_slot, bslot)
        assert bits(r.best_score) == bits(best), b
        assert r.best_inliers[0] == bcnt, b


@pytest.mark.parametrize("solver", [N.SOLVER_HOMOGRAPHY4, N.SOLVER_FUNDAMENTAL7])
def test_pipelined_batches_equal_single_stream(solver, monkeypatch):
    # GCR_VERIFY_PIPE=0 runs generate -> score -> select per batch on one
    # stream; the pipeline must give the same records batch for batch
    if solver == N.SOLVER_HOMOGRAPHY4:
        corr, _, _, thr = S.problem_h(5000, 0.5, seed=SEED)
    else:
        corr, _, _, thr = S.problem_f(10_000, 0.8, seed=SEED)
    prob = CorrProblem(solver, corr)
    p = N.default_params()
    p.scale_residual_thresh, p.seed = thr, SEED
    outs = []
    for pipe in ("1", "0"):
        monkeypatch.setenv("GCR_VERIFY_PIPE", pipe)
        res = (N.BatchResult * 7)()
        N.check(N.lib.gcr_problem_verify_batches(prob.h, C.byref(p), SLOT0, 2048, 7, res, None))
        outs.append([(r.models, r.iterations, r.best_slot, bits(r.best_score).item(), r.best_inliers[0])
                     for r in res])
    assert outs[0] == outs[1]
    assert all(o[2] >= 0 for o in outs[0])


@pytest.mark.parametrize("kind", [N.SOLVER_SIFT22, N.SOLVER_SCALE3, N.SOLVER_SCALE3_ORIGINAL])
def test_chained_batches_equal_unchained(kind, monkeypatch):
    # at 4096 slots consecutive fused launches are chained: each one's spare
    # wave generates the next batch's slots, which the next launch scores
    # instead of generating them in its prologue.  GCR_VERIFY_CHAIN=0 turns
    # that off; records must be identical batch for batch
    f0, f1, thr0, thr1 = _rect_problem(kind)
    prob = Problem(kind, f0, f1)
    p = N.default_params()
    p.scale_residual_thresh, p.orientation_residual_thresh, p.seed = thr0, thr1, SEED
    # GCR_VERIFY_OVERLAP=0 keeps chained launches on one stream (the
    # default alternates two streams, each launch chained to the one two
    # batches ahead)
    outs = []
    for chain, overlap in (("1", "1"), ("1", "0"), ("0", "1")):
        monkeypatch.setenv("GCR_VERIFY_CHAIN", chain)
        monkeypatch.setenv("GCR_VERIFY_OVERLAP", overlap)
        res = (N.BatchResult * 6)()
        N.check(N.lib.gcr_problem_verify_batches(prob.h, C.byref(p), SLOT0, 4096, 6, res, None))
        outs.append([(r.models, r.iterations, r.best_slot, bits(r.best_score).item(), r.best_inliers[0],
                      r.best_inliers[1], bits([r.best_model.h7, r.best_model.h8, r.best_model.alpha,
                                               r.best_model.phi]).tolist()) for r in res])
    assert outs[0] == outs[1] == outs[2]
    assert all(o[2] >= 0 for o in outs[0])


@pytest.mark.parametrize("kind,nslots,nb", [(N.SOLVER_SIFT22, 4096, 70), (N.SOLVER_SCALE3, 4096, 3),
                                            (N.SOLVER_SIFT22, 16384, 18), (N.SOLVER_SIFT22, 1500, 5),
                                            (N.SOLVER_SCALE3, 3000, 67)])
def test_deferred_selection_equals_per_batch(kind, nslots, nb, monkeypatch):
    # verify_batches leaves each fused launch's workgroup bests and models in
    # a ring and reduces a whole ring in one launch (64 batches at 4096 slots,
    # 16 at 16384: 70 and 18 batches cross a ring boundary and end on a partial
    # ring).  GCR_VERIFY_DEFER=0 reduces every batch right after its launch
    # (on one stream); with the ring, chained H = 16 batches alternate two
    # streams (3000 slots: partial workgroups, an odd batch count crossing a
    # ring boundary); the records must be identical batch for batch
    f0, f1, thr0, thr1 = _rect_problem(kind)
    prob = Problem(kind, f0, f1)
    p = N.default_params()
    p.scale_residual_thresh, p.orientation_residual_thresh, p.seed = thr0, thr1, SEED
    outs = []
    for defer in ("1", "0"):
        monkeypatch.setenv("GCR_VERIFY_DEFER", defer)
        res = (N.BatchResult * nb)()
        N.check(N.lib.gcr_problem_verify_batches(prob.h, C.byref(p), SLOT0, nslots, nb, res, None))
        outs.append([(r.models, r.iterations, r.best_slot, bits(r.best_score).item(), r.best_inliers[0],
                      r.best_inliers[1], bits([r.best_model.h7, r.best_model.h8, r.best_model.alpha,
                                               r.best_model.phi]).tolist()) for r in res])
    assert outs[0] == outs[1]
    assert all(o[2] >= 0 for o in outs[0])
    assert len({o[2] for o in outs[0]}) > 1          # distinct batches, distinct bests


@pytest.mark.parametrize("solver,nslots,nb", [(N.SOLVER_HOMOGRAPHY4, 4096, 70), (N.SOLVER_FUNDAMENTAL7, 3712, 30),
                                              (N.SOLVER_FUNDAMENTAL7, 14848, 9), (N.SOLVER_HOMOGRAPHY4, 2048, 3)])
def test_correspondence_deferred_selection_equals_per_batch(solver, nslots, nb, monkeypatch):
    # the pipelined correspondence verify_batches scores batch b into ring set
    # b % R (R = 64 at 4096 homography slots, 23 at 3712 fundamental-matrix
    # slots = 11136 hypotheses) and reduces a whole ring in one launch;
    # GCR_VERIFY_DEFER=0 (two buffer sets, a selection per batch) and the
    # one-stream path must give the same records batch for batch
    if solver == N.SOLVER_HOMOGRAPHY4:
        corr, _, _, thr = S.problem_h(5000, 0.5, seed=SEED)
    else:
        corr, _, _, thr = S.problem_f(10_000, 0.8, seed=SEED)
    prob = CorrProblem(solver, corr)
    p = N.default_params()
    p.scale_residual_thresh, p.seed = thr, SEED
    outs = []
    for defer, pipe in (("1", "1"), ("0", "1"), ("1", "0")):
        monkeypatch.setenv("GCR_VERIFY_DEFER", defer)
        monkeypatch.setenv("GCR_VERIFY_PIPE", pipe)
        res = (N.BatchResult * nb)()
        N.check(N.lib.gcr_problem_verify_batches(prob.h, C.byref(p), SLOT0, nslots, nb, res, None))
        outs.append([(r.models, r.iterations, r.best_slot, bits(r.best_score).item(), r.best_inliers[0])
                     for r in res])
    assert outs[0] == outs[1] == outs[2]
    assert all(o[2] >= 0 for o in outs[0])
    assert len({o[2] for o in outs[0]}) > 1
