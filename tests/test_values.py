"""The product's residual values (csrc/rect.h "values": scale_sq_value /
orient_sq_value, what the kernels evaluate and fold) on the host, bitwise
against the oracle's TWIN-mode restatement of the same formulas, and the
product's glibc decision residuals bitwise against the oracle's GLIBC mode
(the reference) -- including the rare paths: the scale cut, negative / zero /
NaN / huge scales, degenerate rectified directions (the orientation value's
reference-formula fallback: magnitudes outside [2^-900, 2^1000], inf, NaN),
models with |phi| > 16 or NaN, non-identity normalisation.  The device twins
of the same functions are compared with the host bitwise in
tests/test_gpu_parity.py (math ops) and end to end in the GPU parity suite."""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O
from pygcransac import _native as N
from pygcransac import synthetic as S

DP = C.POINTER(C.c_double)


@pytest.fixture(scope="module", autouse=True)
def _built():
    O.build()


def host(solver, cls, f, m7, arith):
    f = np.ascontiguousarray(f, dtype=np.float64)
    out = np.zeros(f.shape[0])
    m = N.RectModel(*[float(v) for v in m7])
    N.check(N.lib.gcr_host_residuals(solver, cls, f.ctypes.data_as(DP), f.shape[0], C.byref(m), arith,
                                     out.ctypes.data_as(DP)))
    return out


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return np.array_equal(a.view(np.uint64), b.view(np.uint64)) or bool(
        np.all((a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))))


def _models(rng, k):
    out = []
    for _ in range(k):
        out.append([0.0, 0.0, 1.0, *rng.normal(scale=3e-4, size=2), rng.uniform(0.1, 3.0), rng.uniform(0, 2 * np.pi)])
    # normalisation, extreme alphas, phi outside the fast range, NaN phi, h7 / h8 large
    out += [[120.0, -40.0, 0.01, 2e-4, -1e-4, 1.3, 0.7],
            [0.0, 0.0, 1.0, 1e-4, 2e-4, 1e-70, 1.0],
            [0.0, 0.0, 1.0, 1e-4, 2e-4, 1e70, 1.0],
            [0.0, 0.0, 1.0, 1e-4, 2e-4, 1.0, 17.5],
            [0.0, 0.0, 1.0, 1e-4, 2e-4, 1.0, -40.0],
            [0.0, 0.0, 1.0, 1e-4, 2e-4, 1.0, float("nan")],
            [0.0, 0.0, 1.0, 0.5, -0.25, 1.0, 2.0],
            [0.0, 0.0, 1.0, -1e-3, 1e-3, 0.8, 3.0]]
    return np.array(out)


def _features(rng, cls, n):
    fs, fo, _, _, _, _ = S.problem_m2(n, n, seed=int(rng.integers(1 << 30)))
    f = (fs if cls == 0 else fo).copy()
    if cls == 0:
        f[:8, 2] = [0.0, -1.0, np.nan, np.inf, 1e-300, 1e300, 5e-324, 1e-12]
        f[8:12, :2] = [[1e6, 1e6], [-1e5, 3e5], [np.nan, 0.0], [0.0, np.inf]]
    else:
        f[:6, 2] = [0.0, np.pi / 2, np.pi, np.nan, np.inf, 1e10]
        f[6:10, :2] = [[1e6, 1e6], [-1e5, 3e5], [np.nan, 0.0], [1e300, -1e300]]
    return f


@pytest.mark.parametrize("solver", [0, 1, 2])
def test_host_values_equal_oracle_twin(solver):
    rng = np.random.default_rng(40 + solver)
    for m7 in _models(rng, 12):
        for cls in ((0, 1) if solver == 2 else (0,)):
            f = _features(rng, cls, 600)
            kind = solver
            got = host(solver, cls, f, m7, 0)
            ref = O.residuals(kind, cls, f, m7, math_mode=O.MATH_TWIN)
            assert same(got, ref), (m7, cls, np.nonzero(got.view(np.uint64) != ref.view(np.uint64))[0][:5])
            gg = host(solver, cls, f, m7, 1)
            gr = O.residuals(kind, cls, f, m7, math_mode=O.MATH_GLIBC)
            assert same(gg, gr), (m7, cls)


def test_orientation_fallback_paths_are_exercised():
    """Directions whose rotated magnitude leaves [2^-900, 2^1000] and models
    with |phi| > 16 take the reference formula with the twin atan2: the value
    then equals round 3's twin residual (PURE_TWIN) exactly."""
    f = np.array([[0.0, 0.0, 0.3], [10.0, 20.0, 1.2], [1e306, 1e306, 0.4], [5.0, 5.0, np.nan]])
    m7 = np.array([0.0, 0.0, 1.0, 1e-4, 2e-4, 1.0, 20.0])          # |phi| > 16: every pair
    got = host(2, 1, f, m7, 0)
    assert same(got, O.residuals(2, 1, f, m7, math_mode=O.MATH_PURE_TWIN))
    # huge coordinates: numer / denom overflow the fast path's range
    m7 = np.array([0.0, 0.0, 1.0, 1e-4, 2e-4, 1.0, 1.0])
    got = host(2, 1, f[2:3], m7, 0)
    assert same(got, O.residuals(2, 1, f[2:3], m7, math_mode=O.MATH_PURE_TWIN))


def test_value_deviation_from_glibc_within_bound():
    """|r_value - r_glibc| inside exact.h's bound on random pairs (the flag
    band's premise), measured per class."""
    rng = np.random.default_rng(9)
    worst = [0.0, 0.0]
    for m7 in _models(rng, 30)[:30]:
        for cls in (0, 1):
            fs, fo, _, _, _, _ = S.problem_m2(800, 800, seed=int(rng.integers(1 << 30)))
            f = fs if cls == 0 else fo
            v = np.sqrt(host(2, cls, f, m7, 0))
            g = np.sqrt(host(2, cls, f, m7, 1))
            ok = np.isfinite(v) & np.isfinite(g)
            dev = np.abs(v[ok] - g[ok])
            bound = 4e-15 + 1e-12 * g[ok] if cls == 0 else np.full(dev.shape, 4e-14)
            assert np.all(dev <= bound)
            rel = dev / np.maximum(g[ok], 1.0)
            worst[cls] = max(worst[cls], float(np.max(rel)) if rel.size else 0.0)
    # exact.h: scale <= 1.0e-15 + 5.2e-16 r, orientation <= 5e-15
    assert worst[0] < 1.6e-15 and worst[1] < 5e-15, worst
