"""Helpers shared by the parity tests: device-resident problems through the C
ABI and an exact restatement of Score finalisation for raw GPU accumulators."""
from __future__ import annotations

import ctypes as C

import numpy as np

from pygcransac import _native as N

KINDS = (N.SOLVER_SCALE3, N.SOLVER_SCALE3_ORIGINAL, N.SOLVER_SIFT22)


def dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Problem:
    def __init__(self, kind, f0, f1=None, device=0):
        self.kind = kind
        self.f0 = np.ascontiguousarray(f0, dtype=np.float64)
        self.f1 = None if f1 is None else np.ascontiguousarray(f1, dtype=np.float64)
        self.ctx = N.context(device)
        h = C.c_void_p()
        rc = N.lib.gcr_problem_create(self.ctx, kind, dp(self.f0), self.f0.shape[0],
                                      dp(self.f1) if self.f1 is not None else None,
                                      0 if self.f1 is None else self.f1.shape[0], C.byref(h))
        N.check(rc)
        self.h = h.value

    def close(self):
        if self.h:
            N.lib.gcr_problem_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def generate(self, seed, slot0, nslots):
        inc = np.zeros(nslots, dtype=np.uint8)
        models = (N.RectModel * nslots)()
        N.check(N.lib.gcr_debug_generate(self.h, seed, slot0, nslots, inc.ctypes.data_as(C.POINTER(C.c_uint8)),
                                         models))
        arr = np.array([[m.x0, m.y0, m.s, m.h7, m.h8, m.alpha, m.phi] for m in models])
        return inc, arr

    def score_raw(self, models7, thr0, thr1=0.0):
        n = len(models7)
        ms = (N.RectModel * n)(*[N.RectModel(*map(float, m)) for m in models7])
        p = N.default_params()
        p.scale_residual_thresh = thr0
        p.orientation_residual_thresh = thr1
        n0 = np.zeros(n, dtype=np.uint32)
        n1 = np.zeros(n, dtype=np.uint32)
        v0, v1, tot = np.zeros(n), np.zeros(n), np.zeros(n)
        u32 = C.POINTER(C.c_uint32)
        N.check(N.lib.gcr_debug_score(self.h, C.byref(p), ms, n, n0.ctypes.data_as(u32), n1.ctypes.data_as(u32),
                                      dp(v0), dp(v1), dp(tot)))
        return n0, n1, v0, v1, tot

    def mask(self, model7, cls, rule, thr0, thr1=0.0, lam=0.0):
        p = N.default_params()
        p.scale_residual_thresh = thr0
        p.orientation_residual_thresh = thr1
        p.spatial_coherence_weight = lam
        n = (self.f0 if cls == 0 else self.f1).shape[0]
        out = np.zeros(n, dtype=np.uint8)
        m = N.RectModel(*map(float, model7))
        N.check(N.lib.gcr_debug_mask(self.h, C.byref(p), C.byref(m), cls, rule,
                                     out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out.astype(bool)


def finish_score(kind, n0, n1, v0, v1, tot, thr0, thr1):
    """MSACScoringFunction::getScore post-processing (MSAC_scoring_function.hpp:108-127)."""
    K = 2 if kind == N.SOLVER_SIFT22 else 1
    m = (2, 2) if K == 2 else (3,)
    T = [(2.25 * thr0) * thr0, (2.25 * thr1) * thr1]
    n = [int(n0), int(n1)]
    v = [float(v0), float(v1)]
    s = float(tot)
    for c in range(K):
        if n[c] < m[c]:
            return dict(counts=[0, 0], values=[0.0, 0.0], value=0.0)
        nv = v[c] / T[c] + float(n[c])
        s -= v[c]
        v[c] = nv
        s += nv
    if K == 1:
        n[1], v[1] = 0, 0.0
    return dict(counts=n, values=v, value=s)


def bits(x):
    return np.asarray(x, dtype=np.float64).view(np.uint64)


u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)


class CorrProblem:
    """A device-resident homography / fundamental-matrix problem (C ABI)."""

    def __init__(self, solver, corr):
        self.solver = solver
        self.c = np.ascontiguousarray(corr, dtype=np.float64)
        h = C.c_void_p()
        N.check(N.lib.gcr_problem_create(N.context(0), solver, dp(self.c), self.c.shape[0], None, 0,
                                         C.byref(h)))
        self.h = h.value

    def close(self):
        if self.h:
            N.lib.gcr_problem_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def generate(self, seed, slot0, n):
        """homography: inc (n,), models (n, 9); fundamental: (n, 3), (n, 3, 9)"""
        per = 3 if self.solver == N.SOLVER_FUNDAMENTAL7 else 1
        inc = np.zeros(n * per, dtype=np.uint8)
        H = np.zeros((n * per, 9))
        N.check(N.lib.gcr_debug_generate_h(self.h, seed, slot0, n, inc.ctypes.data_as(u8p), dp(H)))
        if per == 1:
            return inc, H
        return inc.reshape(n, per), H.reshape(n, per, 9)

    def score(self, models, thr):
        models = np.ascontiguousarray(models, dtype=np.float64)
        n = len(models)
        p = N.default_params()
        p.scale_residual_thresh = thr
        n0 = np.zeros(n, dtype=np.uint32)
        v0, tot = np.zeros(n), np.zeros(n)
        N.check(N.lib.gcr_debug_score_h(self.h, C.byref(p), dp(models), n, n0.ctypes.data_as(u32p), dp(v0), dp(tot)))
        return n0, v0, tot

    def mask(self, model, rule, thr, lam=0.0):
        p = N.default_params()
        p.scale_residual_thresh = thr
        p.spatial_coherence_weight = lam
        out = np.zeros(self.c.shape[0], dtype=np.uint8)
        m = np.ascontiguousarray(model, dtype=np.float64)
        N.check(N.lib.gcr_debug_mask_h(self.h, C.byref(p), dp(m), rule, out.ctypes.data_as(u8p)))
        return out.astype(bool)


# ---------------------------------------------------------------------------
# Thresholds at the boundary between the reference's arithmetic (glibc) and
# the detmath twins: for a pair whose glibc and twin squared residuals differ,
# a threshold whose MSAC T = (2.25 thr) thr lies between them makes the two
# arithmetics decide that pair differently (csrc/exact.h; VERDICT round 3,
# "What's weak" 1).
def msac_T(thr):
    return (2.25 * thr) * thr


def thr_between(a, b):
    """A threshold whose MSAC T lies in [min(a, b), max(a, b)), or None."""
    lo, hi = min(a, b), max(a, b)
    if not (lo < hi):
        return None
    t = float(np.sqrt(lo / 2.25))
    for _ in range(400):
        T = msac_T(t)
        if lo <= T < hi:
            return t
        t = float(np.nextafter(t, np.inf if T < lo else -np.inf))
    return None


def boundary_thresholds(O, kind, f0, f1, thr0, thr1, model, per_class=4, window=0.3, vs=None):
    """(cls, feature, thr0, thr1) cases: for up to `per_class` features of each
    class whose glibc and `vs` r^2 under `model` differ and lie within
    `window` T of the class threshold, the thresholds with that class's moved
    between the two residuals.  `vs`: MATH_TWIN (default: the product's
    values, what the kernels evaluate) or MATH_PURE_TWIN (round 3's twins)."""
    vs = O.MATH_TWIN if vs is None else vs
    out = []
    classes = [(0, f0)] + ([(1, f1)] if kind == N.SOLVER_SIFT22 else [])
    for cls, f in classes:
        g = O.residuals(kind, cls, f, model, math_mode=O.MATH_GLIBC)
        t = O.residuals(kind, cls, f, model, math_mode=vs)
        T = msac_T(thr0 if cls == 0 else thr1)
        idx = np.where((g != t) & np.isfinite(g) & (np.abs(g - T) < window * T))[0]
        for i in idx[:per_class]:
            x = thr_between(g[i], t[i])
            if x is None:
                continue
            th = [thr0, thr1]
            th[cls] = x
            out.append((cls, int(i), th[0], th[1]))
    return out


def first_member_model(O, kind, f0, f1, thr0, thr1, seed, slots=64):
    """The model of the first slot whose hypothesis is valid and scores > 0
    (GLIBC mode, 2-SIFT: the glibc phi): every run with `seed` acts on it --
    it is the first member of the first chunk's chain whatever the threshold
    does to the counts of one pair -- so thresholds built from its residuals
    put a decision of the run itself at the glibc/twin boundary."""
    for s in range(slots):
        inc, m = O.slot(kind, f0, f1, seed, s, math_mode=O.MATH_GLIBC)
        if inc > 101:
            continue
        if kind == N.SOLVER_SIFT22 and not max(abs(m[3]), abs(m[4])) < 1e-3:
            continue
        sc = O.score(kind, f0, f1, m, thr0, thr1, math_mode=O.MATH_GLIBC)
        if sc["value"] > 0:
            return m
    raise AssertionError("no positive valid hypothesis in the first slots")


def best_minimal_model(O, kind, f0, f1, thr0, thr1, seed, budget):
    """The best generated hypothesis of a fixed-budget run (min = max =
    budget iterations, GLIBC mode; 2-SIFT: valid models only, the glibc phi):
    with no LO trials (lo = 0) the final refit fits exactly its MSAC inlier
    lists, so thresholds built from its residuals decide the refit's input."""
    it = s = 0
    best, bv = None, 0.0
    while it < budget:
        inc, m = O.slot(kind, f0, f1, seed, s, math_mode=O.MATH_GLIBC)
        s += 1
        it += inc
        if inc > 101 or (kind == N.SOLVER_SIFT22 and not max(abs(m[3]), abs(m[4])) < 1e-3):
            continue
        v = O.score(kind, f0, f1, m, thr0, thr1, math_mode=O.MATH_GLIBC)["value"]
        if bv < v:
            bv, best = v, m
    return best
