"""Division-free band prefilters of the correspondence scorers at the threshold.

k_score_fm (graph-cut-ransac_amd/csrc/kernels.hip) rejects a (hypothesis,
correspondence) pair before its exact residual when its packed fp32 pre-band
says it cannot be an inlier: transfer error for the homography
(max(|e| - s, 0)^2 > Tb' (|w| + ew)^2), Sampson distance for the fundamental
matrix ((|num| - sn)^2 > T' den_up), both with error bounds from the
problem's largest coordinates.  The split scorers use the fp64 bands h_band
(|e|^2 > Tb w^2) and f_band (num^2 > Tb den).  A band that drops one pair the exact residual accepts changes the
count and the MSAC sum.  These tests place correspondences within one ulp of
the threshold on both sides (bisection on the displacement, evaluated with
the device's own operation order: Python floats are IEEE doubles without FMA
contraction, like -ffp-contract=off) and compare the GPU scores with the
oracle's bitwise, at launch sizes that take every scorer variant.
"""
import math

import numpy as np
import pytest

import oracle_ffi as O
from gcr_testutil import CorrProblem, bits
from pygcransac import _native as N
from pygcransac import synthetic as S


def _f_r2(h, x1, y1, x2, y2):
    """f_sq_sampson (fund.h) in the same operation order."""
    fx0 = (h[0] * x1 + h[1] * y1) + h[2]
    fx1 = (h[3] * x1 + h[4] * y1) + h[5]
    fx2 = (h[6] * x1 + h[7] * y1) + h[8]
    ft0 = (h[0] * x2 + h[3] * y2) + h[6]
    ft1 = (h[1] * x2 + h[4] * y2) + h[7]
    num = (x2 * fx0 + y2 * fx1) + fx2
    den = ((fx0 * fx0 + fx1 * fx1) + ft0 * ft0) + ft1 * ft1
    return (num * num) / den


def _h_r2(h, x1, y1, x2, y2):
    """h_sq_residual (geo.h) in the same operation order."""
    w = (h[6] * x1 + h[7] * y1) + h[8]
    u = ((h[0] * x1 + h[1] * y1) + h[2]) / w
    v = ((h[3] * x1 + h[4] * y1) + h[5]) / w
    du, dv = u - x2, v - y2
    return du * du + dv * dv


def _boundary_corr(solver, models, T, rng, per=80, span=1200.0):
    """Per model, `per` pairs of correspondences straddling r^2 = T: the last
    displacement of a bisection with r^2 <= T and the first with r^2 > T.
    Points x1 are drawn in [0, span)^2."""
    r2f = _f_r2 if solver == N.SOLVER_FUNDAMENTAL7 else _h_r2
    out = []
    for h in models:
        h = [float(v) for v in h]
        for _ in range(per):
            x1, y1 = (float(v) for v in rng.uniform(0, span, size=2))
            if solver == N.SOLVER_FUNDAMENTAL7:
                # foot of a random point on the epipolar line, moved along its normal
                a = (h[0] * x1 + h[1] * y1) + h[2]
                b = (h[3] * x1 + h[4] * y1) + h[5]
                c = (h[6] * x1 + h[7] * y1) + h[8]
                nrm = math.hypot(a, b)
                if nrm == 0.0:
                    continue
                qx, qy = (float(v) for v in rng.uniform(0, span, size=2))
                d = (a * qx + b * qy + c) / nrm
                px, py = qx - d * a / nrm, qy - d * b / nrm
                dx, dy = a / nrm, b / nrm
            else:
                w = (h[6] * x1 + h[7] * y1) + h[8]
                px = ((h[0] * x1 + h[1] * y1) + h[2]) / w
                py = ((h[3] * x1 + h[4] * y1) + h[5]) / w
                ang = rng.uniform(0, 2 * math.pi)
                dx, dy = math.cos(ang), math.sin(ang)
            sgn = 1.0 if rng.random() < 0.5 else -1.0

            def at(t):
                x2, y2 = px + sgn * t * dx, py + sgn * t * dy
                return x2, y2, r2f(h, x1, y1, x2, y2)

            lo, hi = 0.0, math.sqrt(T)
            for _ in range(80):
                if at(hi)[2] > T:
                    break
                lo, hi = hi, 2.0 * hi
            if not at(hi)[2] > T or at(lo)[2] > T:
                continue
            for _ in range(200):
                mid = 0.5 * (lo + hi)
                if mid == lo or mid == hi:
                    break
                if at(mid)[2] > T:
                    hi = mid
                else:
                    lo = mid
            for t in (lo, hi):
                x2, y2, _ = at(t)
                out.append((x1, y1, x2, y2))
    return np.array(out)


@pytest.fixture(scope="module")
def gpu():
    if N.lib.gcr_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    N.context(0)


def _finish(n0, v0, tot, thr, m):
    if int(n0) < m:
        return 0, 0.0
    T = (2.25 * thr) * thr
    return int(n0), (float(tot) - float(v0)) + (float(v0) / T + float(n0))


@pytest.mark.gpu
@pytest.mark.parametrize("solver", [N.SOLVER_HOMOGRAPHY4, N.SOLVER_FUNDAMENTAL7])
def test_band_prefilter_is_conservative_at_the_threshold(gpu, solver):
    rng = np.random.default_rng(77 + solver)
    thr = 0.75
    T = (2.25 * thr) * thr
    if solver == N.SOLVER_FUNDAMENTAL7:
        corr, _, _, _ = S.problem_f(800, 0.3, seed=41)
    else:
        corr, _, _, _ = S.problem_h(800, 0.3, seed=41)
    gen = CorrProblem(solver, corr)
    inc, ms = gen.generate(3, 0, 64)
    models = ms[inc <= 101][:12]
    assert len(models) >= 8
    bc = _boundary_corr(solver, models, T, rng)
    # both sides of the threshold are populated for every model
    r2f = _f_r2 if solver == N.SOLVER_FUNDAMENTAL7 else _h_r2
    side = np.array([r2f(models[0], *map(float, c)) <= T for c in bc[:160]])
    assert 40 < side.sum() < 120
    prob = CorrProblem(solver, bc)
    score_ref = O.f_score if solver == N.SOLVER_FUNDAMENTAL7 else O.h_score
    refs = [score_ref(bc, m, thr) for m in models]
    mmin = 7 if solver == N.SOLVER_FUNDAMENTAL7 else 4
    assert min(r["count"] for r in refs) >= 80           # every model's inlier half
    for nh in (100, 2048, 11136, 16384):                  # H = 4 split, H = 16 feature-major, H = 64 split
        tiled = np.resize(models, (nh, 9))
        n0, v0, tot = prob.score(tiled, thr)
        for i in range(nh):
            ref = refs[i % len(models)]
            cnt, val = _finish(n0[i], v0[i], tot[i], thr, mmin)
            assert cnt == ref["count"], (nh, i)
            assert bits(val) == bits(ref["value"]), (nh, i)


@pytest.mark.gpu
@pytest.mark.parametrize("solver", [N.SOLVER_HOMOGRAPHY4, N.SOLVER_FUNDAMENTAL7])
@pytest.mark.parametrize("span", [20_000.0, 200_000.0])
def test_fp32_preband_is_conservative_at_large_coordinates(gpu, solver, span):
    # the correspondence scorers' packed fp32 pre-bands (Sampson distance,
    # transfer error) carry error bounds scaled by the problem's largest
    # coordinates: correspondences one ulp either side of the threshold far
    # from the origin still score as the oracle
    rng = np.random.default_rng(int(span) + solver)
    thr = 0.75
    T = (2.25 * thr) * thr
    fund = solver == N.SOLVER_FUNDAMENTAL7
    corr, _, _, _ = (S.problem_f if fund else S.problem_h)(800, 0.3, seed=43)
    gen = CorrProblem(solver, corr)
    inc, ms = gen.generate(5, 0, 64)
    models = ms[inc <= 101][:10]
    bc = _boundary_corr(solver, models, T, rng, per=60, span=span)
    prob = CorrProblem(solver, bc)
    refs = [(O.f_score if fund else O.h_score)(bc, m, thr) for m in models]
    assert min(r["count"] for r in refs) >= 60
    for nh in (2048, 11136):                              # the feature-major scorer
        tiled = np.resize(models, (nh, 9))
        n0, v0, tot = prob.score(tiled, thr)
        for i in range(nh):
            ref = refs[i % len(models)]
            cnt, val = _finish(n0[i], v0[i], tot[i], thr, 7 if fund else 4)
            assert cnt == ref["count"], (span, nh, i)
            assert bits(val) == bits(ref["value"]), (span, nh, i)
