"""Known-answer tests of the reference (tests/unit_tests.cpp:13-282), ported to
pin the CPU oracle's restatement of math_utils.hpp and model.h, and the
product's Python model classes (bindings.cpp:329-364)."""
import math

import numpy as np
import pytest

import oracle_ffi as O
import pygcransac

EPS = 1e-9


@pytest.fixture(scope="module")
def L():
    O.build()
    return O.lib()


def _hull(L, pts):
    xy = np.ascontiguousarray(np.asarray(pts, dtype=np.float64).ravel())
    out = np.zeros(2 * len(pts) + 2)
    n = L.oracle_convex_hull(O._dp(xy), len(pts), O._dp(out))
    return sorted(map(tuple, out[: 2 * n].reshape(n, 2)))


def test_collinear_points_positive_case(L):           # unit_tests.cpp:13-21
    assert L.oracle_are_collinear(1, 0, 2, 1, 3, 2, 1e-9) == 1


def test_collinear_points_negative_case(L):           # unit_tests.cpp:23-31
    assert L.oracle_are_collinear(1, 0, 2, 1, 1, 4, 1e-9) == 0


def test_collinearity_is_signed(L):
    # math_utils.hpp:150-154: dist < tol without abs -> the "negative" side counts
    # as collinear (SURVEY finding 0.6); p3 far on the other side of the line:
    assert L.oracle_are_collinear(1, 0, 2, 1, 10, -40, 1e-9) == 1


def test_convex_hull_standard_case(L):                # unit_tests.cpp:37-67
    pts = [(0, 3), (2, 2), (1, 1), (2, 1), (3, 0), (0, 0), (3, 3)]
    assert _hull(L, pts) == sorted([(0, 0), (3, 0), (3, 3), (0, 3)])


def test_convex_hull_degenerate_1d(L):                # unit_tests.cpp:69-80
    h = _hull(L, [(1.45, -5.2)] * 10)
    assert len(h) == 1 and abs(h[0][0] - 1.45) < EPS and abs(h[0][1] + 5.2) < EPS


def test_convex_hull_degenerate_2d(L):                # unit_tests.cpp:82-107
    pts = [(1.45, -5.2), (-3.14, -1.73)] * 5
    assert _hull(L, pts) == sorted([(1.45, -5.2), (-3.14, -1.73)])


@pytest.mark.parametrize("p,inside", [((1, 2), True), ((-1, 2), False), ((1.5, 1.5), True), ((3, 3), True)])
def test_point_in_polygon(L, p, inside):              # unit_tests.cpp:113-148
    sq = np.array([0, 0, 3, 0, 3, 3, 0, 3], dtype=np.float64)
    assert bool(L.oracle_point_in_polygon(p[0], p[1], O._dp(sq), 4)) is inside


def test_line_from_point_and_angle(L):                # unit_tests.cpp:154-178
    l1 = np.zeros(3)
    L.oracle_line_from_point_angle(0.0, 0.0, 0.0, O._dp(l1))
    assert abs(np.dot(l1, [1.0, 0.0, 1.0])) < EPS
    assert abs(abs(np.dot(l1, [-1.0, 1.0, 1.0])) - 1.0) < EPS
    l2 = np.zeros(3)
    L.oracle_line_from_point_angle(1.0, 1.0, math.pi / 2, O._dp(l2))
    x = np.cross(l1, l2)
    assert abs(x[2]) > EPS
    x = x / x[2]
    assert abs(x[0] - 1.0) < EPS and abs(x[1]) < EPS


def test_degrees_to_radians(L):                       # unit_tests.cpp:180-188
    assert abs(L.oracle_deg2rad(90.0) - math.pi / 2) < EPS
    assert abs(L.oracle_rad2deg(math.pi / 2) - 90.0) < EPS
    assert abs(L.oracle_rad2deg(L.oracle_deg2rad(90.0)) - 90.0) < EPS


@pytest.mark.parametrize("a,exp", [(-math.pi / 2, 1.5 * math.pi), (0.7861, 0.7861), (0.0, 0.0),
                                   (2.7 * math.pi, 0.7 * math.pi), (-math.pi, math.pi)])
def test_clip_angle(L, a, exp):                       # unit_tests.cpp:190-203
    assert abs(L.oracle_clip_angle(a) - exp) < EPS


@pytest.mark.parametrize("a,b,exp", [(0.0, 0.0, 0.0), (-math.pi / 2, 0.0, math.pi / 2),
                                     (-3.48 * math.pi, 7.41 * math.pi, 0.89 * math.pi),
                                     (0.25 * math.pi, 1.25 * math.pi, math.pi)])
def test_min_angle_diff(L, a, b, exp):                # unit_tests.cpp:205-217
    assert abs(L.oracle_min_angle_diff(a, b) - exp) < EPS


@pytest.mark.parametrize("a,b,exp", [(0.0, 0.0, 0.0), (-math.pi / 2, 0.0, math.pi / 2),
                                     (0.52 * math.pi, 1.49 * math.pi, 0.03 * math.pi),
                                     (1.49 * math.pi, 0.52 * math.pi, 0.03 * math.pi),
                                     (-3.48 * math.pi, 5.60 * math.pi, 0.08 * math.pi),
                                     (0.25 * math.pi, 1.25 * math.pi, 0.0)])
def test_lines_angles_diff(L, a, b, exp):             # unit_tests.cpp:219-233
    assert abs(L.oracle_lines_angles_diff(a, b) - exp) < EPS


def test_n_choose_2(L):                               # unit_tests.cpp:239-243
    assert (L.oracle_nchoose2(6), L.oracle_nchoose2(1), L.oracle_nchoose2(0)) == (15, 0, 0)


def _roundtrip(rectified_scale, unrectified_scale, rectified_angle, unrectified_angle, rect_pt, unrect_pt):
    udx, udy, uds, udt = 82.4, -12.3, 1.13, 0.56
    ds = unrectified_scale(udx, udy, uds)
    dt = unrectified_angle(udx, udy, udt)
    dx, dy = unrect_pt(udx, udy)
    uds_c = rectified_scale(dx, dy, ds)
    udt_c = rectified_angle(dx, dy, dt)
    udx_c, udy_c = rect_pt(dx, dy)
    for a, b in [(udx, udx_c), (udy, udy_c), (uds, uds_c), (udt, udt_c)]:
        assert abs(a - b) < 1e-12


def test_rectifying_homography_roundtrip_oracle(L):   # unit_tests.cpp:249-282
    m = np.array([0, 0, 1, 0.0001, 0.0002, 1, 0], dtype=np.float64)

    def op(k):
        return lambda x, y, v: L.oracle_model_op(O._dp(m), k, x, y, v, O.MATH_GLIBC)

    def pt(rect):
        def f(x, y):
            out = np.zeros(2)
            L.oracle_model_point(O._dp(m), rect, x, y, O._dp(out))
            return tuple(out)
        return f

    _roundtrip(op(0), op(1), op(2), op(3), pt(1), pt(0))


def test_rectifying_homography_roundtrip_python_classes():
    model = pygcransac.RectifyingHomography()
    model.h7 = 0.0001
    model.h8 = 0.0002
    _roundtrip(model.rectifiedScale, model.unrectifiedScale, model.rectifiedAngle, model.unrectifiedAngle,
               model.rectifiedPoint, model.unrectifiedPoint)


def test_python_model_methods_match_oracle_bitwise(L):
    rng = np.random.default_rng(0)
    for _ in range(200):
        h7, h8 = rng.normal(scale=2e-4, size=2)
        x0, y0, s = rng.normal(scale=50, size=2).tolist() + [float(rng.uniform(0.5, 2))]
        m7 = np.array([x0, y0, s, h7, h8, 0.5, 0.3])
        pm = pygcransac.RectifyingHomography()
        pm.x0, pm.y0, pm.s, pm.h7, pm.h8 = x0, y0, s, h7, h8
        x, y, v = rng.uniform(0, 1500), rng.uniform(0, 1500), rng.uniform(0.1, 6)
        for k, fn in enumerate([pm.rectifiedScale, pm.unrectifiedScale, pm.rectifiedAngle, pm.unrectifiedAngle]):
            assert fn(x, y, v) == L.oracle_model_op(O._dp(m7), k, x, y, v, O.MATH_GLIBC)
        for rect, fn in [(1, pm.rectifiedPoint), (0, pm.unrectifiedPoint)]:
            out = np.zeros(2)
            L.oracle_model_point(O._dp(m7), rect, x, y, O._dp(out))
            assert fn(x, y) == tuple(out)
        H = np.zeros(9)
        L.oracle_get_homography(O._dp(m7), O._dp(H))
        assert np.array_equal(pm.getHomography().ravel(), H)
