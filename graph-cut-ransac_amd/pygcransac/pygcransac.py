"""pygcransac -- drop-in Python API of yuvalnis/graph-cut-ransac, MI355X engine.

Surface mirrors ``src/pygcransac/src/bindings.cpp:315-396`` of the reference:
three functions with the same positional/keyword arguments, defaults, input
validation messages and return tuples, and the five model classes with the
same names, inheritance, attributes and methods.  Extensions are keyword-only
(``seed``, ``confidence``, ``device``, ``batch_slots``, ``return_stats``).

Compute goes through the C ABI in ``include/gcr.h`` (libgcr.so: HIP kernels for
gfx950 plus the host engine).  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import math
import numbers

import numpy as np

from . import _native as N

__all__ = [
    "NormalizingTransform",
    "RectifyingHomography",
    "ScaleBasedRectifyingHomography",
    "OrientationBasedRectifyingHomography",
    "SIFTRectifyingHomography",
    "findRectifyingHomographyScaleOnly",
    "findRectifyingHomographyScaleOnlyOriginal",
    "findRectifyingHomographySIFT",
    "findHomography",
    "findFundamentalMatrix",
]

_TWO_PI = 2.0 * math.pi


# ----------------------------------------------------------- model classes --
class _F64:
    """double data member with pybind11 def_readwrite semantics."""

    def __set_name__(self, owner, name):
        self.name = "_" + name

    def __get__(self, obj, objtype=None):
        if obj is None:
            return self
        return obj.__dict__[self.name]

    def __set__(self, obj, value):
        if type(value) is float:                     # the common case, no ABC checks
            obj.__dict__[self.name] = value
            return
        if isinstance(value, (str, bytes)) or not isinstance(value, (numbers.Real, np.floating, np.integer)):
            raise TypeError(f"incompatible type for double attribute: {type(value).__name__}")
        obj.__dict__[self.name] = float(value)


def _cpow(x, y):
    """glibc pow() itself (numpy's SIMD power is not glibc, math.pow raises)."""
    return _libm.pow(x, y)


def _clip_angle(a):
    # math_utils.hpp:78-88 (std::fmod, then + 2pi if negative)
    if math.isinf(a) or math.isnan(a):
        return math.nan
    a = math.fmod(a, _TWO_PI)
    if a < 0.0:
        a += _TWO_PI
    return a


def _atan2(y, x):
    return math.atan2(y, x)


_libm = C.CDLL("libm.so.6")
_libm.pow.argtypes = [C.c_double, C.c_double]
_libm.pow.restype = C.c_double
_libm.sincos.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
_libm.sincos.restype = None


def _sincos(t):
    """glibc sincos: the reference (GCC -O3) fuses model.h's adjacent
    std::cos/std::sin calls into sincos, which differs from separate sin/cos
    in ~0.1% of arguments."""
    s, c = C.c_double(), C.c_double()
    _libm.sincos(t, C.byref(s), C.byref(c))
    return s.value, c.value


class NormalizingTransform:
    """model.h:42-120"""
    x0 = _F64()
    y0 = _F64()
    s = _F64()

    def __init__(self):
        self.x0 = 0.0
        self.y0 = 0.0
        self.s = 1.0

    def _fields(self):
        return {k: getattr(self, k) for k in ("x0", "y0", "s")}

    def __repr__(self):
        inner = ", ".join(f"{k}={v!r}" for k, v in self._fields().items())
        return f"{type(self).__name__}({inner})"


class RectifyingHomography(NormalizingTransform):
    """model.h:122-227 (+ the pybind11 lambdas at bindings.cpp:335-353)."""
    h7 = _F64()
    h8 = _F64()

    def __init__(self):
        super().__init__()
        self.h7 = 0.0
        self.h8 = 0.0

    def _fields(self):
        d = super()._fields()
        d.update(h7=self.h7, h8=self.h8)
        return d

    def rectifiedScale(self, dx, dy, ds):
        return float(ds) * _cpow(-self.h7 * float(dx) - self.h8 * float(dy) + 1.0, -3.0)

    def unrectifiedScale(self, udx, udy, uds):
        return float(uds) * _cpow(self.h7 * float(udx) + self.h8 * float(udy) + 1.0, -3.0)

    def rectifiedAngle(self, x, y, angle):
        x, y, angle = float(x), float(y), float(angle)
        st, ct = _sincos(angle)
        numer = (-x * st + y * ct) * self.h7 + st
        denom = (x * st - y * ct) * self.h8 + ct
        return _clip_angle(_atan2(numer, denom))

    def unrectifiedAngle(self, x, y, angle):
        x, y, angle = float(x), float(y), float(angle)
        st, ct = _sincos(angle)
        numer = (x * st - y * ct) * self.h7 + st
        denom = (-x * st + y * ct) * self.h8 + ct
        return _clip_angle(_atan2(numer, denom))

    def rectifiedPoint(self, x, y):
        x, y = float(x), float(y)
        w = -self.h7 * x - self.h8 * y + 1.0
        with np.errstate(all="ignore"):
            return (float(np.float64(x) / w), float(np.float64(y) / w))

    def unrectifiedPoint(self, x, y):
        x, y = float(x), float(y)
        w = self.h7 * x + self.h8 * y + 1.0
        with np.errstate(all="ignore"):
            return (float(np.float64(x) / w), float(np.float64(y) / w))

    def getHomography(self):
        # N.inverse() * [[1,0,0],[0,1,0],[h7,h8,1]] * N / H22 with Eigen's
        # 3x3 cofactor inverse, evaluated in IEEE double like the C++ code.
        s, x0, y0 = self.s, self.x0, self.y0
        Nm = [s, 0.0, -s * x0, 0.0, s, -s * y0, 0.0, 0.0, 1.0]
        Hn = [1.0, 0.0, 0.0, 0.0, 1.0, 0.0, self.h7, self.h8, 1.0]

        def cof(i, j):
            i1, i2, j1, j2 = (i + 1) % 3, (i + 2) % 3, (j + 1) % 3, (j + 2) % 3
            return Nm[i1 * 3 + j1] * Nm[i2 * 3 + j2] - Nm[i1 * 3 + j2] * Nm[i2 * 3 + j1]

        with np.errstate(all="ignore"):
            det = (cof(0, 0) * Nm[0] + cof(1, 0) * Nm[3]) + cof(2, 0) * Nm[6]
            invdet = float(np.float64(1.0) / det)
            Ni = [cof(c, r) * invdet for r in range(3) for c in range(3)]
            T = [(Ni[i * 3] * Hn[j] + Ni[i * 3 + 1] * Hn[3 + j]) + Ni[i * 3 + 2] * Hn[6 + j]
                 for i in range(3) for j in range(3)]
            R = [(T[i * 3] * Nm[j] + T[i * 3 + 1] * Nm[3 + j]) + T[i * 3 + 2] * Nm[6 + j]
                 for i in range(3) for j in range(3)]
            d = np.float64(R[8])
            return np.array([np.float64(v) / d for v in R], dtype=np.float64).reshape(3, 3)


class ScaleBasedRectifyingHomography(RectifyingHomography):
    """model.h:229-234"""
    alpha = _F64()

    def __init__(self):
        super().__init__()
        self.alpha = 1.0

    def _fields(self):
        d = super()._fields()
        d.update(alpha=self.alpha)
        return d


class OrientationBasedRectifyingHomography(RectifyingHomography):
    """model.h:236-241"""
    phi = _F64()

    def __init__(self):
        super().__init__()
        self.phi = 0.0

    def _fields(self):
        d = super()._fields()
        d.update(phi=self.phi)
        return d


class SIFTRectifyingHomography(ScaleBasedRectifyingHomography, OrientationBasedRectifyingHomography):
    """model.h:243-246"""


# --------------------------------------------------------------- helpers ---
def _as_features(arr):
    """py::array_t<double> conversion (forcecast) + flat C-contiguous buffer."""
    try:
        a = np.asarray(arr, dtype=np.float64)
    except (TypeError, ValueError) as exc:
        raise TypeError(f"incompatible function arguments: cannot convert to float64 array ({exc})") from None
    return a


def _as_size_t(v, name):
    if type(v) is int and 0 <= v <= 0xFFFFFFFFFFFFFFFF:
        return v
    if isinstance(v, (bool, np.bool_)):
        v = int(v)
    if not isinstance(v, (numbers.Integral, np.integer)) or v < 0:
        raise TypeError(f"incompatible function arguments: {name} must be a non-negative integer")
    if int(v) > 0xFFFFFFFFFFFFFFFF:
        raise TypeError(f"incompatible function arguments: {name} does not fit size_t")
    return int(v)


def _as_double(v, name):
    if type(v) is float:
        return v
    if isinstance(v, (str, bytes)) or not isinstance(v, (numbers.Real, np.floating, np.integer)):
        raise TypeError(f"incompatible function arguments: {name} must be a float")
    return float(v)


def _params(thr0, thr1, lam, min_it, max_it, lo, seed, confidence, batch_slots):
    p = N.default_params()
    p.scale_residual_thresh = _as_double(thr0, "scale_residual_thresh")
    p.orientation_residual_thresh = _as_double(thr1, "orientation_residual_thresh")
    p.spatial_coherence_weight = _as_double(lam, "spatial_coherence_weight")
    p.min_iteration_number = _as_size_t(min_it, "min_iteration_number")
    p.max_iteration_number = _as_size_t(max_it, "max_iteration_number")
    p.max_local_optimization_number = _as_size_t(lo, "max_local_optimization_number")
    p.seed = _as_size_t(seed, "seed")
    p.confidence = _as_double(confidence, "confidence")
    p.batch_slots = _as_size_t(batch_slots, "batch_slots") & 0xFFFFFFFF
    return p


_DP, _U8P = C.POINTER(C.c_double), C.POINTER(C.c_uint8)


def _dp(a):
    return C.cast(a.ctypes.data, _DP)


def _u8(a):
    return C.cast(a.ctypes.data, _U8P)


def _fill(model, m: N.RectModel, sift: bool):
    # the engine's doubles straight into the model's slots (_F64 stores
    # Python floats under "_" + name; ctypes double fields read as floats)
    d = model.__dict__
    d["_x0"], d["_y0"], d["_s"] = m.x0, m.y0, m.s
    d["_h7"], d["_h8"], d["_alpha"] = m.h7, m.h8, m.alpha
    if sift:
        d["_phi"] = m.phi
    return model


def _validate_scale_only(features):
    f = _as_features(features)
    if f.ndim != 2:
        raise ValueError("Number of dimensions must be 2.")
    n, cols = f.shape
    if n < 3 or cols != 3:
        raise ValueError(f"Features should be an array with 3 columns and at least 3 rows. "
                         f"It has {cols} columns and {n} rows.")
    return np.ascontiguousarray(f)


def _scale_only(original, features, scale_residual_thresh, spatial_coherence_weight, min_iteration_number,
                max_iteration_number, max_local_optimization_number, seed, confidence, device, batch_slots,
                return_stats):
    f = _validate_scale_only(features)
    p = _params(scale_residual_thresh, 2.0, spatial_coherence_weight, min_iteration_number, max_iteration_number,
                max_local_optimization_number, seed, confidence, batch_slots)
    n = f.shape[0]
    mask = np.zeros(n, dtype=np.uint8)
    H = np.zeros(9, dtype=np.float64)
    m = N.RectModel()
    st = N.Stats()
    ctx = N.context(device)
    rc = N.lib.gcr_rect_scale_only(ctx, f.ctypes.data, n, C.byref(p), 1 if original else 0, mask.ctypes.data,
                                   H.ctypes.data, C.byref(m), C.byref(st))
    num_inliers = N.check(rc)
    inliers = mask.view(bool)
    extra = (st.as_dict(),) if return_stats else ()
    if num_inliers == 0:
        return (None, inliers) + extra
    model = _fill(ScaleBasedRectifyingHomography(), m, sift=False)
    return (H.reshape(3, 3), inliers, model) + extra


# -------------------------------------------------------------- entry points
def findRectifyingHomographyScaleOnly(features, scale_residual_thresh, spatial_coherence_weight=0.0,
                                      min_iteration_number=10000, max_iteration_number=10000,
                                      max_local_optimization_number=50, *, seed=0, confidence=0.95, device=None,
                                      batch_slots=0, return_stats=False):
    """3-SIFT scale-only rectification (bindings.cpp:19-98, 366-374).

    Returns ``(H, inliers, ScaleBasedRectifyingHomography)`` or ``(None, inliers)``
    when no model is found.
    """
    return _scale_only(False, features, scale_residual_thresh, spatial_coherence_weight, min_iteration_number,
                       max_iteration_number, max_local_optimization_number, seed, confidence, device, batch_slots,
                       return_stats)


def findRectifyingHomographyScaleOnlyOriginal(features, scale_residual_thresh, spatial_coherence_weight=0.0,
                                              min_iteration_number=10000, max_iteration_number=10000,
                                              max_local_optimization_number=50, *, seed=0, confidence=0.95,
                                              device=None, batch_slots=0, return_stats=False):
    """Original-parametrisation 3-SIFT solver (bindings.cpp:100-179, 376-384)."""
    return _scale_only(True, features, scale_residual_thresh, spatial_coherence_weight, min_iteration_number,
                       max_iteration_number, max_local_optimization_number, seed, confidence, device, batch_slots,
                       return_stats)


def findRectifyingHomographySIFT(scale_features, orientation_features, scale_residual_thresh,
                                 orientation_residual_thresh, spatial_coherence_weight=0.0,
                                 min_iteration_number=10000, max_iteration_number=10000,
                                 max_local_optimization_number=50, *, seed=0, confidence=0.95, device=None,
                                 batch_slots=0, return_stats=False):
    """Hybrid 2+2 SIFT rectification (bindings.cpp:181-311, 386-396).

    Returns ``(H, scale_inliers, orientation_inliers, SIFTRectifyingHomography)``
    or ``(None, scale_inliers, orientation_inliers, None)``.
    """
    fs = _as_features(scale_features)
    fo = _as_features(orientation_features)
    if fs.ndim != 2 or fo.ndim != 2:
        raise ValueError("Number of dimensions must be 2.")
    ns, cs = fs.shape
    no, co = fo.shape
    if ns < 2 or cs != 3:
        raise ValueError(f"Scale features should be an array with 3 columns and at least 2 rows. "
                         f"It has {cs} columns and {ns} rows.")
    if no < 2 or co != 3:
        raise ValueError(f"Orientation features should be an array with 3 columns and at least 2 rows. "
                         f"It has {co} columns and {no} rows.")
    fs = np.ascontiguousarray(fs)
    fo = np.ascontiguousarray(fo)
    p = _params(scale_residual_thresh, orientation_residual_thresh, spatial_coherence_weight, min_iteration_number,
                max_iteration_number, max_local_optimization_number, seed, confidence, batch_slots)
    ms = np.zeros(ns, dtype=np.uint8)
    mo = np.zeros(no, dtype=np.uint8)
    H = np.zeros(9, dtype=np.float64)
    m = N.RectModel()
    st = N.Stats()
    ctx = N.context(device)
    rc = N.lib.gcr_rect_sift(ctx, fs.ctypes.data, ns, fo.ctypes.data, no, C.byref(p), ms.ctypes.data,
                             mo.ctypes.data, H.ctypes.data, C.byref(m), C.byref(st))
    num_inliers = N.check(rc)
    s_in, o_in = ms.view(bool), mo.view(bool)
    extra = (st.as_dict(),) if return_stats else ()
    if num_inliers == 0:
        return (None, s_in, o_in, None) + extra
    model = _fill(SIFTRectifyingHomography(), m, sift=True)
    return (H.reshape(3, 3), s_in, o_in, model) + extra


def grid_cell_sizes(correspondences, h1, w1, h2, w2, neighborhood_size):
    """Cell sizes of the neighbourhood grid over (x1, y1, x2, y2): each image
    extent divided by `neighborhood_size` cells (upstream GC-RANSAC's
    GridNeighborhoodGraph<4> over {w1, h1, w2, h2} / cells).  An image size
    <= 0 (unknown) is replaced by the correspondences' extent along that axis
    (max coordinate + 1, at least 1 px)."""
    k = float(neighborhood_size)
    sizes = [float(v) for v in (w1, h1, w2, h2)]
    known = [v > 0.0 and math.isfinite(v) for v in sizes]
    if not all(known):
        f = np.asarray(correspondences, dtype=np.float64)
        for col in range(4):
            if known[col]:
                continue
            if not f.size:
                sizes[col] = 1.0
                continue
            c = f[:, col]
            top = float(c.max())                    # NaN / inf present: the finite values only
            if not math.isfinite(top):
                fin = c[np.isfinite(c)]
                top = float(fin.max()) if fin.size else None
            sizes[col] = max(1.0, top + 1.0) if top is not None else 1.0
    return [v / k for v in sizes]


def grid_params(correspondences, h1, w1, h2, w2, neighborhood_size, from_data=True):
    """(cell_number, cell sizes or None) of gcr_params' neighbourhood grid.
    from_data=False leaves an unknown image size's cells at 0 for the engine
    to take from the data (the same values, computed natively)."""
    cells = _as_size_t(neighborhood_size, "neighborhood_size")
    if cells > 0xFFFFFFFF:
        raise ValueError("neighborhood_size does not fit 32 bits")
    if not cells:
        return cells, None
    if from_data:
        return cells, grid_cell_sizes(correspondences, h1, w1, h2, w2, cells)
    k = float(cells)
    return cells, [float(v) / k if float(v) > 0.0 and math.isfinite(float(v)) else 0.0 for v in (w1, h1, w2, h2)]


def _set_grid(p, correspondences, h1, w1, h2, w2, neighborhood_size):
    cells, sizes = grid_params(correspondences, h1, w1, h2, w2, neighborhood_size)
    p.cell_number = cells
    if cells:
        p.cell_size[:] = sizes


def _correspondence_call(entry, correspondences, h1, w1, h2, w2, probabilities, threshold, conf,
                         spatial_coherence_weight, max_iters, min_iters, sampler, lo_number, seed, device,
                         batch_slots, return_stats, min_rows, neighborhood_size):
    for name, v in (("h1", h1), ("w1", w1), ("h2", h2), ("w2", w2)):
        _as_double(v, name)
    if probabilities is not None and len(probabilities) != 0:
        raise ValueError("Only the uniform sampler is supported; probabilities must be empty.")
    if _as_size_t(sampler, "sampler") != 0:
        raise ValueError(f"Unsupported sampler {sampler}: only 0 (uniform) is supported.")
    f = _as_features(correspondences)
    if f.ndim != 2:
        raise ValueError("Number of dimensions must be 2.")
    n, cols = f.shape
    if n < min_rows or cols != 4:
        raise ValueError(f"Correspondences should be an array with 4 columns and at least {min_rows} rows. "
                         f"It has {cols} columns and {n} rows.")
    f = np.ascontiguousarray(f)
    p = _params(threshold, 2.0, spatial_coherence_weight, min_iters, max_iters, lo_number, seed, conf, batch_slots)
    _set_grid(p, f, h1, w1, h2, w2, neighborhood_size)
    mask = np.zeros(n, dtype=np.uint8)
    M = np.zeros(9, dtype=np.float64)
    st = N.Stats()
    ctx = N.context(device)
    rc = entry(ctx, f.ctypes.data, n, C.byref(p), mask.ctypes.data, M.ctypes.data, C.byref(st))
    num_inliers = N.check(rc)
    inliers = mask.view(bool)
    extra = (st.as_dict(),) if return_stats else ()
    if num_inliers == 0:
        return (None, inliers) + extra
    return (M.reshape(3, 3), inliers) + extra


def findHomography(correspondences, h1, w1, h2, w2, probabilities=None, threshold=1.0, conf=0.99,
                   spatial_coherence_weight=0.975, max_iters=10000, min_iters=50, sampler=0, lo_number=50, *,
                   neighborhood_size=8, seed=0, device=None, batch_slots=0, return_stats=False):
    """4-point homography with graph-cut LO -- an EXTENSION (SURVEY.md §8(f)
    row 3): this fork has no homography estimator (finding 0.1); the argument
    names and order follow upstream pygcransac's findHomography.

    ``correspondences`` is (N, 4) float64: x1, y1, x2, y2.  ``h1, w1, h2, w2``
    are the image sizes: the graph-cut's neighbourhood grid over (x1, y1, x2,
    y2) has ``neighborhood_size`` cells along each axis (cell sizes w1/k, h1/k,
    w2/k, h2/k; a size <= 0 is taken from the data's extent), and
    ``spatial_coherence_weight`` (lambda) weighs its pairwise terms in every
    graph-cut labeling (GCRANSAC.h:759-870); ``neighborhood_size=0`` or
    lambda = 0 gives the empty grid.  ``sampler`` must be 0 (uniform) and
    ``probabilities`` empty.  ``threshold`` is the inlier threshold in pixels
    of the second image (MSAC threshold 2.25 * threshold, as the rectification
    solvers).

    Returns ``(H, inliers)`` with H (3, 3) and H[2, 2] = 1, or ``(None, inliers)``.
    """
    return _correspondence_call(N.lib.gcr_find_homography, correspondences, h1, w1, h2, w2, probabilities,
                                threshold, conf, spatial_coherence_weight, max_iters, min_iters, sampler, lo_number,
                                seed, device, batch_slots, return_stats, 4, neighborhood_size)


def findFundamentalMatrix(correspondences, h1, w1, h2, w2, probabilities=None, threshold=1.0, conf=0.99,
                          spatial_coherence_weight=0.975, max_iters=10000, min_iters=50, sampler=0, lo_number=50,
                          *, neighborhood_size=8, seed=0, device=None, batch_slots=0, return_stats=False):
    """7-point fundamental matrix with graph-cut LO -- an EXTENSION like
    findHomography (same arguments, the same neighbourhood grid; upstream
    pygcransac's findFundamentalMatrix order).  The residual is the Sampson distance in pixels; a sample yields up
    to three models, each scored.

    Returns ``(F, inliers)`` with F (3, 3), unit Frobenius norm and
    x2^T F x1 = 0, or ``(None, inliers)``.
    """
    return _correspondence_call(N.lib.gcr_find_fundamental_matrix, correspondences, h1, w1, h2, w2, probabilities,
                                threshold, conf, spatial_coherence_weight, max_iters, min_iters, sampler, lo_number,
                                seed, device, batch_slots, return_stats, 7, neighborhood_size)
