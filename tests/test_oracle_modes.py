"""The oracle's two math modes agree: GLIBC mode (the reference's own libm for
log / pow / atan2) and TWIN mode (detmath, bit-identical on host and GPU).
GPU parity is asserted bitwise against TWIN mode (test_gpu_parity.py); this
file ties TWIN mode back to the reference's arithmetic: identical inlier
masks and run statistics, models within the north_star 1e-6 relative bound."""
import numpy as np
import pytest

import oracle_ffi as O
from pygcransac import synthetic as S

# bounded budgets keep the CPU suite fast; the adaptive stop still applies
KW = dict(min_it=100, max_it=1500, seed=7)


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300))) if a.size else 0.0


def _run_stats(r):
    st = r["stats"]
    return {k: st[k] for k in ("iteration_number", "local_optimization_number", "graph_cut_number")}


def _models(r):
    m = r["model"]
    return np.array([m[k] for k in sorted(m)])


@pytest.fixture(scope="module", autouse=True)
def _built():
    O.build()


@pytest.mark.parametrize("original", [False, True])
@pytest.mark.parametrize("n,seed", [(300, 1), (1200, 2)])
def test_scale_only_glibc_and_twin_agree(original, n, seed):
    f, _, thr = S.problem_m1(n, seed=seed)
    g = O.rect_scale_only(f, thr, original=original, math_mode=O.MATH_GLIBC, **KW)
    t = O.rect_scale_only(f, thr, original=original, math_mode=O.MATH_TWIN, **KW)
    assert np.array_equal(g["mask"], t["mask"])
    assert g["num_inliers"] == t["num_inliers"]
    assert _run_stats(g) == _run_stats(t)
    assert _rel(_models(t), _models(g)) <= 1e-6
    assert _rel(t["H"], g["H"]) <= 1e-6


@pytest.mark.parametrize("n,seed", [(300, 3), (1000, 4)])
def test_sift_glibc_and_twin_agree(n, seed):
    fs, fo, _, _, ts, to = S.problem_m2(n, n, seed=seed)
    g = O.rect_sift(fs, fo, ts, to, math_mode=O.MATH_GLIBC, **KW)
    t = O.rect_sift(fs, fo, ts, to, math_mode=O.MATH_TWIN, **KW)
    assert np.array_equal(g["scale_mask"], t["scale_mask"])
    assert np.array_equal(g["orientation_mask"], t["orientation_mask"])
    assert _run_stats(g) == _run_stats(t)
    assert _rel(_models(t), _models(g)) <= 1e-6
    assert _rel(t["H"], g["H"]) <= 1e-6


def test_twin_residuals_track_glibc_within_few_ulp():
    # per-feature residuals r of many random models: |r_twin - r_glibc| stays at
    # a few ulp of O(1) (detmath bounds: log <= 0.77, pow_m3 < 2, atan2 <= 1.8
    # ulp); measured max 8.9e-16 with ~20 % of residuals differing at all
    fs, fo, _, _, _, _ = S.problem_m2(400, 400, seed=9)
    rng = np.random.default_rng(5)
    worst = 0.0
    for _ in range(40):
        m = np.array([0, 0, 1, *rng.normal(scale=2e-4, size=2), rng.uniform(0.2, 2), rng.uniform(0, np.pi)])
        for kind, cls, f in [(0, 0, fs), (2, 1, fo)]:
            g = np.sqrt(O.residuals(kind, cls, f, m, math_mode=O.MATH_GLIBC))
            t = np.sqrt(O.residuals(kind, cls, f, m, math_mode=O.MATH_TWIN))
            assert np.array_equal(np.isfinite(g), np.isfinite(t))
            ok = np.isfinite(g)
            worst = max(worst, float(np.max(np.abs(t[ok] - g[ok]))))
    assert worst <= 4e-15
