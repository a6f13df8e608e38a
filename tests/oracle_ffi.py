"""ctypes bindings to the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker, never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "_build", "liboracle.so")

MATH_GLIBC, MATH_TWIN, MATH_PURE_TWIN = 0, 1, 2
SAMPLER_PHILOX, SAMPLER_FAITHFUL = 0, 1
KIND_SCALE3, KIND_SCALE3_ORIGINAL, KIND_SIFT22 = 0, 1, 2


class OracleParams(C.Structure):
    _fields_ = [
        ("thr0", C.c_double), ("thr1", C.c_double), ("spatial_coherence_weight", C.c_double),
        ("min_iteration_number", C.c_uint64), ("max_iteration_number", C.c_uint64),
        ("max_local_optimization_number", C.c_uint64), ("confidence", C.c_double),
        ("seed", C.c_uint64), ("math_mode", C.c_int32), ("sampler", C.c_int32),
        ("cell_size", C.c_double * 4), ("cell_number", C.c_uint64),
    ]


class OracleStats(C.Structure):
    _fields_ = [
        ("iteration_number", C.c_uint64), ("local_optimization_number", C.c_uint64),
        ("graph_cut_number", C.c_uint64), ("slots", C.c_uint64), ("hypotheses", C.c_uint64),
        ("score", C.c_double), ("seconds", C.c_double),
        ("near_ties", C.c_uint64), ("near_tie_flips", C.c_uint64),
    ]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        dp, u8p, u64p = C.POINTER(C.c_double), C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)
        L.oracle_rect_scale_only.argtypes = [dp, C.c_size_t, C.POINTER(OracleParams), C.c_int, u8p, dp, dp,
                                             C.POINTER(OracleStats)]
        L.oracle_rect_sift.argtypes = [dp, C.c_size_t, dp, C.c_size_t, C.POINTER(OracleParams), u8p, u8p, dp, dp,
                                       C.POINTER(OracleStats)]
        L.oracle_slot.argtypes = [C.c_int, dp, C.c_size_t, dp, C.c_size_t, C.c_uint64, C.c_uint64, C.c_int, dp]
        L.oracle_score.argtypes = [C.c_int, dp, C.c_size_t, dp, C.c_size_t, dp, C.c_double, C.c_double, C.c_int,
                                   u64p, dp, dp, u8p, u8p]
        L.oracle_residuals.argtypes = [C.c_int, C.c_int, dp, C.c_size_t, dp, C.c_int, dp]
        L.oracle_sample.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                    C.c_uint32, u64p]
        L.oracle_philox.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.oracle_philox.restype = None
        L.oracle_fit_nonminimal.argtypes = [C.c_int, dp, C.c_size_t, dp, C.c_size_t, u64p, C.c_size_t, u64p,
                                            C.c_size_t, C.c_int, dp]
        L.oracle_hot_batch.argtypes = [C.c_int, dp, C.c_size_t, dp, C.c_size_t, C.c_double, C.c_double, C.c_uint64,
                                       C.c_uint64, C.c_uint64, C.c_int, C.c_int, dp, dp]
        L.oracle_hot_batch.restype = C.c_int64
        L.oracle_find_homography.argtypes = [dp, C.c_size_t, C.POINTER(OracleParams), u8p, dp,
                                             C.POINTER(OracleStats)]
        L.oracle_h_slot.argtypes = [dp, C.c_size_t, C.c_uint64, C.c_uint64, dp]
        L.oracle_h_score.argtypes = [dp, C.c_size_t, dp, C.c_double, u64p, dp, u8p]
        L.oracle_h_residuals.argtypes = [dp, C.c_size_t, dp, dp]
        L.oracle_find_fundamental.argtypes = L.oracle_find_homography.argtypes
        u32p = C.POINTER(C.c_uint32)
        L.oracle_bk_energy.argtypes = [C.c_size_t, dp, u32p, dp, C.c_size_t, u8p, dp]
        L.oracle_grid_edges.argtypes = [dp, C.c_size_t, C.c_size_t, dp, C.c_uint64, u32p, C.c_size_t]
        L.oracle_grid_edges.restype = C.c_size_t
        L.oracle_f_slot.argtypes = [dp, C.c_size_t, C.c_uint64, C.c_uint64, dp, C.POINTER(C.c_int)]
        L.oracle_f_score.argtypes = L.oracle_h_score.argtypes
        L.oracle_f_residuals.argtypes = L.oracle_h_residuals.argtypes
        L.oracle_f_fit.argtypes = L.oracle_h_fit.argtypes
        L.oracle_h_fit.argtypes = [dp, C.c_size_t, u64p, C.c_size_t, dp]
        for name in ["oracle_clip_angle", "oracle_deg2rad", "oracle_rad2deg"]:
            getattr(L, name).argtypes = [C.c_double]
            getattr(L, name).restype = C.c_double
        for name in ["oracle_min_angle_diff", "oracle_lines_angles_diff"]:
            getattr(L, name).argtypes = [C.c_double, C.c_double]
            getattr(L, name).restype = C.c_double
        L.oracle_nchoose2.argtypes = [C.c_uint64]
        L.oracle_nchoose2.restype = C.c_uint64
        L.oracle_are_collinear.argtypes = [C.c_double] * 7
        L.oracle_line_from_point_angle.argtypes = [C.c_double, C.c_double, C.c_double, dp]
        L.oracle_line_from_point_angle.restype = None
        L.oracle_convex_hull.argtypes = [dp, C.c_size_t, dp]
        L.oracle_point_in_polygon.argtypes = [C.c_double, C.c_double, dp, C.c_size_t]
        L.oracle_model_op.argtypes = [dp, C.c_int, C.c_double, C.c_double, C.c_double, C.c_int]
        L.oracle_model_op.restype = C.c_double
        L.oracle_model_point.argtypes = [dp, C.c_int, C.c_double, C.c_double, dp]
        L.oracle_model_point.restype = None
        L.oracle_get_homography.argtypes = [dp, dp]
        L.oracle_get_homography.restype = None
        L.oracle_gauss3.argtypes = [dp, dp]
        L.oracle_lstsq3.argtypes = [dp, C.c_size_t, dp, dp]
        L.oracle_weighted_mode.argtypes = [dp, dp, C.c_size_t, C.c_double]
        L.oracle_weighted_mode.restype = C.c_double
        L.oracle_set_qr_order.argtypes = [C.c_int]
        _lib = L
    return _lib


QR_BLOCKED, QR_FROZEN = 0, 1


class qr_order:
    """Context manager: run the oracle's least-squares fits in `order`
    (QR_FROZEN = the frozen sequential reduction order, never changed to follow
    the product; QR_BLOCKED = the engine's blocked order, the default)."""

    def __init__(self, order):
        self.order = order

    def __enter__(self):
        self.prev = lib().oracle_set_qr_order(self.order)
        return self

    def __exit__(self, *exc):
        lib().oracle_set_qr_order(self.prev)
        return False


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def params(thr0, thr1=0.0, lam=0.0, min_it=10000, max_it=10000, lo=50, confidence=0.95, seed=0,
           math_mode=MATH_TWIN, sampler=SAMPLER_PHILOX, cell_size=(0.0, 0.0, 0.0, 0.0), cell_number=0):
    """cell_size / cell_number: the H / F neighbourhood grid over (x1, y1, x2,
    y2) (0 cells = the empty grid of the reference's entry points)."""
    return OracleParams(thr0, thr1, lam, min_it, max_it, lo, confidence, seed, math_mode, sampler,
                        (C.c_double * 4)(*map(float, cell_size)), int(cell_number))


def model7(m):
    return np.array([m["x0"], m["y0"], m["s"], m["h7"], m["h8"], m["alpha"], m["phi"]], dtype=np.float64)


def _model_dict(v):
    return dict(x0=v[0], y0=v[1], s=v[2], h7=v[3], h8=v[4], alpha=v[5], phi=v[6])


def _stats_dict(st):
    return {k: getattr(st, k) for k, _ in OracleStats._fields_}


def rect_scale_only(features, thr, original=False, **kw):
    f = _f64(features)
    n = f.shape[0]
    mask = np.zeros(n, dtype=np.uint8)
    H = np.zeros(9)
    m = np.zeros(7)
    st = OracleStats()
    p = params(thr, **kw)
    r = lib().oracle_rect_scale_only(_dp(f), n, C.byref(p), int(original),
                                     mask.ctypes.data_as(C.POINTER(C.c_uint8)), _dp(H), _dp(m), C.byref(st))
    if r < 0:
        raise RuntimeError("oracle failed")
    return dict(num_inliers=r, mask=mask.astype(bool), H=H.reshape(3, 3), model=_model_dict(m),
                stats=_stats_dict(st))


def rect_sift(scale_features, orientation_features, thr_s, thr_o, **kw):
    fs, fo = _f64(scale_features), _f64(orientation_features)
    ms = np.zeros(fs.shape[0], dtype=np.uint8)
    mo = np.zeros(fo.shape[0], dtype=np.uint8)
    H = np.zeros(9)
    m = np.zeros(7)
    st = OracleStats()
    p = params(thr_s, thr_o, **kw)
    r = lib().oracle_rect_sift(_dp(fs), fs.shape[0], _dp(fo), fo.shape[0], C.byref(p),
                               ms.ctypes.data_as(C.POINTER(C.c_uint8)), mo.ctypes.data_as(C.POINTER(C.c_uint8)),
                               _dp(H), _dp(m), C.byref(st))
    if r < 0:
        raise RuntimeError("oracle failed")
    return dict(num_inliers=r, scale_mask=ms.astype(bool), orientation_mask=mo.astype(bool),
                H=H.reshape(3, 3), model=_model_dict(m), stats=_stats_dict(st))


def slot(kind, f0, f1, seed, slot_index, math_mode=MATH_TWIN):
    f0 = _f64(f0)
    f1 = _f64(f1) if f1 is not None else None
    m = np.zeros(7)
    inc = lib().oracle_slot(kind, _dp(f0), f0.shape[0], _dp(f1) if f1 is not None else None,
                            0 if f1 is None else f1.shape[0], seed, slot_index, math_mode, _dp(m))
    return inc, m


def score(kind, f0, f1, model, thr0, thr1=0.0, math_mode=MATH_TWIN, want_masks=False):
    f0 = _f64(f0)
    f1 = _f64(f1) if f1 is not None else None
    counts = np.zeros(2, dtype=np.uint64)
    values = np.zeros(2)
    value = np.zeros(1)
    m0 = np.zeros(f0.shape[0], dtype=np.uint8) if want_masks else None
    m1 = np.zeros(f1.shape[0], dtype=np.uint8) if (want_masks and f1 is not None) else None
    u8 = C.POINTER(C.c_uint8)
    lib().oracle_score(kind, _dp(f0), f0.shape[0], _dp(f1) if f1 is not None else None,
                       0 if f1 is None else f1.shape[0], _dp(_f64(model)), thr0, thr1, math_mode,
                       counts.ctypes.data_as(C.POINTER(C.c_uint64)), _dp(values), _dp(value),
                       m0.ctypes.data_as(u8) if m0 is not None else None,
                       m1.ctypes.data_as(u8) if m1 is not None else None)
    out = dict(counts=counts, values=values, value=float(value[0]))
    if want_masks:
        out["masks"] = (m0.astype(bool), None if m1 is None else m1.astype(bool))
    return out


def residuals(kind, cls, f, model, math_mode=MATH_TWIN):
    f = _f64(f)
    r2 = np.zeros(f.shape[0])
    lib().oracle_residuals(kind, cls, _dp(f), f.shape[0], _dp(_f64(model)), math_mode, _dp(r2))
    return r2


def sample(seed, index, sub, stream, cls, n, m):
    out = np.zeros(m, dtype=np.uint64)
    r = lib().oracle_sample(seed, index, sub, stream, cls, n, m, out.ctypes.data_as(C.POINTER(C.c_uint64)))
    if r != 0:
        raise RuntimeError("sample budget exhausted")
    return out


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().oracle_philox(c, k, o)
    return list(o)


def fit_nonminimal(kind, f0, f1, idx0, idx1=None, math_mode=MATH_TWIN):
    f0 = _f64(f0)
    f1 = _f64(f1) if f1 is not None else None
    i0 = np.ascontiguousarray(np.asarray(idx0, dtype=np.uint64))
    i1 = np.ascontiguousarray(np.asarray(idx1 if idx1 is not None else [], dtype=np.uint64))
    m = np.zeros(7)
    u64 = C.POINTER(C.c_uint64)
    ok = lib().oracle_fit_nonminimal(kind, _dp(f0), f0.shape[0], _dp(f1) if f1 is not None else None,
                                     0 if f1 is None else f1.shape[0], i0.ctypes.data_as(u64), len(i0),
                                     i1.ctypes.data_as(u64), len(i1), math_mode, _dp(m))
    return (m if ok else None)


def find_homography(corr, thr, **kw):
    c = _f64(corr)
    n = c.shape[0]
    mask = np.zeros(n, dtype=np.uint8)
    H = np.zeros(9)
    st = OracleStats()
    p = params(thr, **kw)
    r = lib().oracle_find_homography(_dp(c), n, C.byref(p), mask.ctypes.data_as(C.POINTER(C.c_uint8)), _dp(H),
                                     C.byref(st))
    if r < 0:
        raise RuntimeError("oracle failed")
    return dict(num_inliers=r, mask=mask.astype(bool), H=H.reshape(3, 3), stats=_stats_dict(st))


def h_slot(corr, seed, slot):
    c = _f64(corr)
    m = np.zeros(9)
    inc = lib().oracle_h_slot(_dp(c), c.shape[0], seed, slot, _dp(m))
    return inc, m


def h_score(corr, model9, thr, want_mask=False):
    c = _f64(corr)
    cnt = C.c_uint64()
    val = C.c_double()
    mask = np.zeros(c.shape[0], dtype=np.uint8) if want_mask else None
    lib().oracle_h_score(_dp(c), c.shape[0], _dp(_f64(model9)), thr, C.byref(cnt), C.byref(val),
                         mask.ctypes.data_as(C.POINTER(C.c_uint8)) if want_mask else None)
    out = dict(count=int(cnt.value), value=val.value)
    if want_mask:
        out["mask"] = mask.astype(bool)
    return out


def h_residuals(corr, model9):
    c = _f64(corr)
    r2 = np.zeros(c.shape[0])
    lib().oracle_h_residuals(_dp(c), c.shape[0], _dp(_f64(model9)), _dp(r2))
    return r2


def h_fit(corr, idx):
    c = _f64(corr)
    i = np.ascontiguousarray(np.asarray(idx, dtype=np.uint64))
    m = np.zeros(9)
    ok = lib().oracle_h_fit(_dp(c), c.shape[0], i.ctypes.data_as(C.POINTER(C.c_uint64)), len(i), _dp(m))
    return m if ok else None


def find_fundamental(corr, thr, **kw):
    c = _f64(corr)
    n = c.shape[0]
    mask = np.zeros(n, dtype=np.uint8)
    H = np.zeros(9)
    st = OracleStats()
    p = params(thr, **kw)
    r = lib().oracle_find_fundamental(_dp(c), n, C.byref(p), mask.ctypes.data_as(C.POINTER(C.c_uint8)), _dp(H),
                                     C.byref(st))
    if r < 0:
        raise RuntimeError("oracle failed")
    return dict(num_inliers=r, mask=mask.astype(bool), H=H.reshape(3, 3), stats=_stats_dict(st))


def f_slot(corr, seed, slot):
    """(inc, models (k, 9)) of one outer-iteration slot of the 7-point solver."""
    c = _f64(corr)
    m = np.zeros(27)
    k = C.c_int()
    inc = lib().oracle_f_slot(_dp(c), c.shape[0], seed, slot, _dp(m), C.byref(k))
    return inc, m.reshape(3, 9)[:k.value].copy()


def f_score(corr, model9, thr, want_mask=False):
    c = _f64(corr)
    cnt = C.c_uint64()
    val = C.c_double()
    mask = np.zeros(c.shape[0], dtype=np.uint8) if want_mask else None
    lib().oracle_f_score(_dp(c), c.shape[0], _dp(_f64(model9)), thr, C.byref(cnt), C.byref(val),
                         mask.ctypes.data_as(C.POINTER(C.c_uint8)) if want_mask else None)
    out = dict(count=int(cnt.value), value=val.value)
    if want_mask:
        out["mask"] = mask.astype(bool)
    return out


def f_residuals(corr, model9):
    c = _f64(corr)
    r2 = np.zeros(c.shape[0])
    lib().oracle_f_residuals(_dp(c), c.shape[0], _dp(_f64(model9)), _dp(r2))
    return r2


def f_fit(corr, idx):
    c = _f64(corr)
    i = np.ascontiguousarray(np.asarray(idx, dtype=np.uint64))
    m = np.zeros(9)
    ok = lib().oracle_f_fit(_dp(c), c.shape[0], i.ctypes.data_as(C.POINTER(C.c_uint64)), len(i), _dp(m))
    return m if ok else None


def hot_batch(kind, f0, f1, thr0, thr1, seed, slot0, nslots, sampler=SAMPLER_FAITHFUL, math_mode=MATH_GLIBC):
    """Single-thread CPU hot path (sample+solve+score) over nslots slots."""
    f0 = _f64(f0)
    f1 = _f64(f1) if f1 is not None else None
    sec = np.zeros(1)
    best = np.zeros(1)
    n = lib().oracle_hot_batch(kind, _dp(f0), f0.shape[0], _dp(f1) if f1 is not None else None,
                               0 if f1 is None else f1.shape[0], thr0, thr1, seed, slot0, nslots, sampler,
                               math_mode, _dp(sec), _dp(best))
    return int(n), float(sec[0]), float(best[0])


def bk_energy(unary, edges, pair):
    """BK restatement over an energy: unary (n, 2) = E_i(0), E_i(1); edges
    (m, 2); pair (m, 4) = E(00), E(01), E(10), E(11).  Returns (seg (n,) bool,
    True = SINK, flow)."""
    u = _f64(np.asarray(unary).reshape(-1, 2))
    e = np.ascontiguousarray(np.asarray(edges, dtype=np.uint32).reshape(-1, 2))
    pr = _f64(np.asarray(pair).reshape(-1, 4))
    seg = np.zeros(u.shape[0], dtype=np.uint8)
    flow = C.c_double()
    lib().oracle_bk_energy(u.shape[0], _dp(u), e.ctypes.data_as(C.POINTER(C.c_uint32)), _dp(pr), e.shape[0],
                           seg.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(flow))
    return seg.astype(bool), flow.value


def grid_edges(points, cell_size, cell_number):
    """The neighbourhood grid's edge list in labeling()'s order, (m, 2)."""
    pts = _f64(points)
    cs = _f64(np.asarray(cell_size, dtype=np.float64))
    n, d = pts.shape
    m = lib().oracle_grid_edges(_dp(pts), n, d, _dp(cs), int(cell_number), None, 0)
    out = np.zeros((max(m, 1), 2), dtype=np.uint32)
    lib().oracle_grid_edges(_dp(pts), n, d, _dp(cs), int(cell_number), out.ctypes.data_as(C.POINTER(C.c_uint32)), m)
    return out[:m]


def score_less(kind, f0, f1, ma, mb, thr0, thr1=0.0, math_mode=MATH_TWIN):
    """The run loop's `score(ma) < score(mb)` (GCRANSAC.h:440) in math_mode:
    (decision, near_tie, value_order) -- GLIBC compares glibc scores, TWIN the
    value scores with the near-tie rule (csrc/exact.h ScoreBound)."""
    f0 = _f64(f0)
    f1 = _f64(f1) if f1 is not None else None
    L = lib()
    dp = C.POINTER(C.c_double)
    L.oracle_score_less.restype = C.c_int
    L.oracle_score_less.argtypes = [C.c_int, dp, C.c_size_t, dp, C.c_size_t, dp, dp, C.c_double, C.c_double, C.c_int]
    r = L.oracle_score_less(kind, _dp(f0), f0.shape[0], _dp(f1) if f1 is not None else None,
                            0 if f1 is None else f1.shape[0], _dp(_f64(ma)), _dp(_f64(mb)), thr0, thr1, math_mode)
    return bool(r & 1), bool(r & 2), bool(r & 4)
