"""The product's non-minimal fits (host_fit.cpp + qr3.h, behind
gcr_host_fit_nonminimal) against the oracle's independent restatement,
bitwise: LO-sized systems (plain sequential sums) and final-refit-sized
hybrid systems (thousands of vanishing-point pair rows, blocked sums)."""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O
from pygcransac import _native as N
from pygcransac import synthetic as S


def _product_fit(kind, f0, f1, i0, i1):
    f0 = np.ascontiguousarray(f0, dtype=np.float64)
    f1 = None if f1 is None else np.ascontiguousarray(f1, dtype=np.float64)
    a0 = np.ascontiguousarray(i0, dtype=np.uint32)
    a1 = np.ascontiguousarray(i1 if i1 is not None else [], dtype=np.uint32)
    m = N.RectModel()
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    u32 = C.POINTER(C.c_uint32)
    rc = N.lib.gcr_host_fit_nonminimal(kind, dp(f0), f0.shape[0], dp(f1) if f1 is not None else None,
                                       0 if f1 is None else f1.shape[0], a0.ctypes.data_as(u32), len(a0),
                                       a1.ctypes.data_as(u32), len(a1), C.byref(m))
    assert rc >= 0
    return None if rc == 0 else np.array([m.x0, m.y0, m.s, m.h7, m.h8, m.alpha, m.phi])


@pytest.fixture(scope="module", autouse=True)
def _built():
    O.build()


@pytest.mark.parametrize("kind", [N.SOLVER_SCALE3, N.SOLVER_SCALE3_ORIGINAL])
@pytest.mark.parametrize("k", [3, 4, 14, 300, 1023, 1024, 1025, 4000])
def test_scale_fit_matches_oracle_bitwise(kind, k):
    f, truth, _ = S.problem_m1(10000, seed=11 + k)
    rng = np.random.default_rng(k)
    idx = np.sort(rng.choice(np.flatnonzero(truth), size=k, replace=False))
    got = _product_fit(kind, f, None, idx, None)
    exp = O.fit_nonminimal(kind, f, None, idx)
    if exp is None:
        assert got is None
    else:
        assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))


@pytest.mark.parametrize("ks,ko", [(2, 2), (3, 2), (14, 14), (60, 45), (500, 46), (800, 120), (2000, 260),
                                   (0, 300), (3, 600)])
def test_sift_fit_matches_oracle_bitwise(ks, ko):
    # ko = 46 -> 1035 pair rows (blocked order starts); 260 -> 33 670 rows:
    # >= 32768 rows take the double-double Gram path (gram.h); (0, 300): no
    # scale rows, the rank-deficient pivot branch
    fs, fo, ts, to, _, _ = S.problem_m2(5000, 3000, seed=ks + ko)
    rng = np.random.default_rng(ks * 7 + ko)
    i0 = np.sort(rng.choice(np.flatnonzero(ts), size=ks, replace=False))
    i1 = np.sort(rng.choice(np.flatnonzero(to), size=ko, replace=False))
    got = _product_fit(N.SOLVER_SIFT22, fs, fo, i0, i1)
    exp = O.fit_nonminimal(N.SOLVER_SIFT22, fs, fo, i0, i1)
    if exp is None:
        assert got is None
    else:
        assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))
        # and within the frozen pin's tolerance of the sequential Householder order
        with O.qr_order(O.QR_FROZEN):
            frz = O.fit_nonminimal(N.SOLVER_SIFT22, fs, fo, i0, i1)
        assert np.all(np.abs(got - frz) <= 1e-6 * np.maximum(np.abs(frz), 1e-12))


def test_weighted_mode_matches_oracle_including_ties():
    # findWeightedMode (two_sift.hpp:354-394): the first maximum in
    # unordered_map iteration order decides ties; the product accumulates in
    # arrays and rebuilds only the map's key order (first occurrences)
    import ctypes as C

    import numpy as np

    import oracle_ffi as O
    from pygcransac import _native as N

    dp = C.POINTER(C.c_double)
    bw = 0.5 * np.pi / 180.0
    rng = np.random.default_rng(17)
    cases = []
    for n in (1, 2, 14, 91, 500, 2500, 6000):
        a = rng.uniform(0, np.pi, n)
        cases.append((a, np.full(n, 1.0 / n)))                       # equal weights: many ties
        cases.append((np.round(a / bw) * bw + rng.uniform(-0.2, 0.2, n) * bw, rng.uniform(0, 1, n)))
    cases.append((np.array([0.1, 0.1 + 1e5, -3.0, 7e3]), np.ones(4) / 4))   # sparse bins
    cases.append((np.array([0.2, np.nan, 0.3]), np.array([0.5, 0.25, 0.25])))
    cases.append((np.zeros(0), np.zeros(0)))
    for a, w in cases:
        a = np.ascontiguousarray(a, dtype=np.float64)
        w = np.ascontiguousarray(w, dtype=np.float64)
        got = N.lib.gcr_host_weighted_mode(a.ctypes.data_as(dp), w.ctypes.data_as(dp), a.size, bw)
        ref = O.lib().oracle_weighted_mode(a.ctypes.data_as(dp), w.ctypes.data_as(dp), a.size, bw)
        assert np.array_equal(np.float64(got).view(np.uint64), np.float64(ref).view(np.uint64)) or \
            (np.isnan(got) and np.isnan(ref)), (a.size, got, ref)
