"""The summary replay (the default, engine.cpp replay_summaries + summary.hip)
against the per-slot replay it replaced (GCR_REPLAY=slots): every chunk is
summarised on the device to its prefix-maximum chain, totals and last live
hypothesis, and the host walks only the chain (GCRANSAC.h:286-531 acts only on
strict new bests).  Both must give identical runs -- masks, model bits,
iteration / hypothesis / LO / graph-cut counts, slots, score -- for every
estimator, fixed and adaptive budgets, tiny chunks, a one-member summary cap
(every chunk overflows and is continued on the device) and with the next chunk
issued ahead or not, and one-part blocks summarised by the fused one-wave
kernel (k_sum_one) or the three launches.  The oracle parity of the default
path is tested everywhere else (golden, end-to-end, bench-config tests)."""
import ctypes as C

import numpy as np
import pytest

from gcr_testutil import CorrProblem, Problem, bits
from pygcransac import _native as N
from pygcransac import synthetic as S

pytestmark = pytest.mark.gpu

SOLVERS = [N.SOLVER_SCALE3, N.SOLVER_SCALE3_ORIGINAL, N.SOLVER_SIFT22, N.SOLVER_HOMOGRAPHY4,
           N.SOLVER_FUNDAMENTAL7]


def _data(kind):
    if kind == N.SOLVER_SIFT22:
        fs, fo, _, _, ts, to = S.problem_m2(1500, 1300, seed=61)
        return fs, fo, ts, to
    if kind == N.SOLVER_HOMOGRAPHY4:
        c, _, _, thr = S.problem_h(2500, 0.6, seed=62)
        return c, None, thr, 0.0
    if kind == N.SOLVER_FUNDAMENTAL7:
        c, _, _, thr = S.problem_f(2500, 0.6, seed=63)
        return c, None, thr, 0.0
    f, _, thr = S.problem_m1(2500, seed=64 + kind)
    return f, None, thr, 0.0


def _run(kind, budget, monkeypatch, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    f0, f1, thr0, thr1 = _data(kind)
    prob = CorrProblem(kind, f0) if kind >= N.SOLVER_HOMOGRAPHY4 else Problem(kind, f0, f1)
    p = N.default_params()
    p.scale_residual_thresh, p.orientation_residual_thresh, p.seed = thr0, thr1, 11
    if budget == "fixed":                  # 65536-slot chunks, the last one cut by the budget
        p.min_iteration_number = p.max_iteration_number = 300_000
    elif budget == "adaptive":             # 256 -> 1024 -> ... slots, adaptive termination
        p.min_iteration_number, p.max_iteration_number, p.confidence = 0, 10**7, 0.99
    elif budget == "tiny":                 # 37-slot chunks
        p.min_iteration_number, p.max_iteration_number, p.confidence, p.batch_slots = 50, 5000, 0.999, 37
    elif budget == "floor":                # an iteration floor past the adaptive stop
        p.min_iteration_number, p.max_iteration_number, p.confidence = 150_000, 10**7, 0.95
    m0 = np.zeros(f0.shape[0], np.uint8)
    m1 = np.zeros(0 if f1 is None else f1.shape[0], np.uint8)
    H = np.zeros(9)
    model = N.RectModel()
    st = N.Stats()
    u8 = C.POINTER(C.c_uint8)
    n = N.check(N.lib.gcr_problem_run(prob.h, C.byref(p), m0.ctypes.data_as(u8),
                                      m1.ctypes.data_as(u8) if f1 is not None else None,
                                      H.ctypes.data_as(C.POINTER(C.c_double)), C.byref(model), C.byref(st)))
    for k in env:
        monkeypatch.delenv(k)
    return (n, m0.tobytes(), m1.tobytes(), bits(H).tobytes(), st.iteration_number, st.hypotheses,
            st.local_optimization_number, st.graph_cut_number, bits(st.score).tobytes(), st.slots)


@pytest.mark.parametrize("kind", SOLVERS)
@pytest.mark.parametrize("budget", ["fixed", "adaptive", "tiny", "floor"])
def test_summary_replay_equals_slot_replay(kind, budget, monkeypatch):
    ref = _run(kind, budget, monkeypatch, {"GCR_REPLAY": "slots"})
    assert ref[0] > 0 and ref[4] > 0
    assert _run(kind, budget, monkeypatch, {}) == ref
    # every summary holds one member: the chain continues on the device
    assert _run(kind, budget, monkeypatch, {"GCR_SUMMARY_CAP": "1"}) == ref
    # no chunk issued ahead of the replay
    assert _run(kind, budget, monkeypatch, {"GCR_PREFETCH": "0", "GCR_SUMMARY_CAP": "3"}) == ref
    # one-part blocks through the three-launch summary instead of k_sum_one
    assert _run(kind, budget, monkeypatch, {"GCR_SUMMARY_ONE": "0"}) == ref
    assert _run(kind, budget, monkeypatch, {"GCR_SUMMARY_ONE": "0", "GCR_SUMMARY_CAP": "1"}) == ref


def test_slot_replay_after_speculative_chunks_on_recycled_workspace(monkeypatch):
    """An adaptive F run can return with a speculative chunk still running on
    the side stream; the next problem reuses the workspace (last in, first
    out).  The per-slot replay and the upload of the next problem must wait
    for it (engine.cpp await_spec) instead of racing it on set 0's buffers."""
    kind = N.SOLVER_FUNDAMENTAL7
    ref = _run(kind, "adaptive", monkeypatch, {"GCR_REPLAY": "slots"})
    for _ in range(3):
        assert _run(kind, "adaptive", monkeypatch, {}) == ref
        assert _run(kind, "adaptive", monkeypatch, {"GCR_REPLAY": "slots"}) == ref


def _run_m(kind, seed, outliers, monkeypatch, env):
    """An adaptive 0.99 run of a larger M1 / M2 problem with LO on (50
    trials), so several small-scored chunks run on the side stream while the
    replay stream scores LO trials and refits."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if kind == N.SOLVER_SIFT22:
        f0, f1, _, _, thr0, thr1 = S.problem_m2(3000, 3000, outliers, seed=seed)
    else:
        f0, _, thr0 = S.problem_m1(6000, outliers, seed=seed)
        f1, thr1 = None, 0.0
    prob = Problem(kind, f0, f1)
    p = N.default_params()
    p.scale_residual_thresh, p.orientation_residual_thresh, p.seed = thr0, thr1, seed
    p.min_iteration_number, p.max_iteration_number, p.confidence = 0, 10**7, 0.99
    m0 = np.zeros(f0.shape[0], np.uint8)
    m1 = np.zeros(0 if f1 is None else f1.shape[0], np.uint8)
    H = np.zeros(9)
    model = N.RectModel()
    st = N.Stats()
    u8 = C.POINTER(C.c_uint8)
    n = N.check(N.lib.gcr_problem_run(prob.h, C.byref(p), m0.ctypes.data_as(u8),
                                      m1.ctypes.data_as(u8) if f1 is not None else None,
                                      H.ctypes.data_as(C.POINTER(C.c_double)), C.byref(model), C.byref(st)))
    for k in env:
        monkeypatch.delenv(k)
    prob.close()
    return (n, m0.tobytes(), m1.tobytes(), bits(H).tobytes(), st.iteration_number, st.hypotheses,
            st.local_optimization_number, st.graph_cut_number, bits(st.score).tobytes(), st.slots)


@pytest.mark.parametrize("kind,outliers", [(N.SOLVER_SCALE3, 0.8), (N.SOLVER_SIFT22, 0.75)])
def test_small_chunks_on_side_stream_do_not_race_lo_scoring(kind, outliers, monkeypatch):
    """small-scored chunks (<= 256 slots, the split
    scorer) issued speculatively on the side stream must not share the split
    scorer's scratch with the LO trials / refit scored on the replay stream
    (engine.cpp Workspace::cs_vals).  Tiny first chunks keep every chunk of
    the run small-scored; the result must equal the run without any chunk
    issued ahead, and the per-slot replay."""
    for seed in (3, 4, 5):
        ref = _run_m(kind, seed, outliers, monkeypatch, {"GCR_PREFETCH": "0", "GCR_FIRST_CHUNK": "8"})
        assert ref[0] > 0 and ref[6] > 0
        for _ in range(2):
            assert _run_m(kind, seed, outliers, monkeypatch, {"GCR_FIRST_CHUNK": "8"}) == ref
        assert _run_m(kind, seed, outliers, monkeypatch, {"GCR_FIRST_CHUNK": "8", "GCR_CHUNK_CAP": "0"})[:5] == \
            ref[:5]
        assert _run_m(kind, seed, outliers, monkeypatch, {"GCR_REPLAY": "slots"}) == ref
