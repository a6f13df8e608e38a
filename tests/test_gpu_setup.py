"""Problem setup (engine.cpp make_problem): one parallel pass fills the host
classes, the pinned staging image and the column maxima, and the feature upload
stays queued on the context's stream when gcr_problem_create returns (the side
stream waits on its event; the next problem on a recycled workspace waits before
restaging).  Problems created back to back -- destroyed unrun, or alive
together on one context -- must run exactly as a problem created alone."""
import ctypes as C

import numpy as np
import pytest

from gcr_testutil import CorrProblem, Problem, bits
from pygcransac import _native as N
from test_gpu_summary import _data

pytestmark = pytest.mark.gpu


def _make(kind, f0, f1):
    return CorrProblem(kind, f0) if kind >= N.SOLVER_HOMOGRAPHY4 else Problem(kind, f0, f1)


def _run(prob, kind, f0, f1, thr0, thr1):
    p = N.default_params()
    p.scale_residual_thresh, p.orientation_residual_thresh, p.seed = thr0, thr1, 5
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
    return (n, m0.tobytes(), m1.tobytes(), bits(H).tobytes(), st.iteration_number, st.hypotheses,
            st.local_optimization_number, bits(st.score).tobytes())


@pytest.mark.parametrize("kind", [N.SOLVER_SIFT22, N.SOLVER_SCALE3, N.SOLVER_FUNDAMENTAL7])
def test_back_to_back_problems_run_as_alone(kind):
    f0, f1, thr0, thr1 = _data(kind)
    alone = _make(kind, f0, f1)
    ref = _run(alone, kind, f0, f1, thr0, thr1)
    alone.close()
    assert ref[0] > 0
    # created and destroyed without a run (its upload may still be queued),
    # then the problem proper on the recycled workspace
    other = f0[::-1].copy()
    for _ in range(3):
        junk = _make(kind, other, None if f1 is None else f1[::-1].copy())
        junk.close()
        prob = _make(kind, f0, f1)
        assert _run(prob, kind, f0, f1, thr0, thr1) == ref
        prob.close()
    # several problems alive on one context, run out of creation order
    probs = [_make(kind, f0, f1) for _ in range(3)]
    for prob in reversed(probs):
        assert _run(prob, kind, f0, f1, thr0, thr1) == ref
    for prob in probs:
        prob.close()


def test_nonfinite_features_run_deterministically():
    """A NaN and an infinity among the features (the parallel fill's column
    maxima become +inf, which disables the packed pre-bands' rejections):
    two runs of the same data on fresh problems agree."""
    f0, f1, thr0, thr1 = _data(N.SOLVER_SIFT22)
    f0 = f0.copy()
    f0[17, 0] = np.nan
    f0[401, 2] = np.inf
    a = _make(N.SOLVER_SIFT22, f0, f1)
    r1 = _run(a, N.SOLVER_SIFT22, f0, f1, thr0, thr1)
    a.close()
    b = _make(N.SOLVER_SIFT22, f0, f1)
    assert _run(b, N.SOLVER_SIFT22, f0, f1, thr0, thr1) == r1
    b.close()
