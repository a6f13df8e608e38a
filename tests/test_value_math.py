"""The primitives of the product's residual values (csrc/detmath.h, round 4),
host side: the table log (dm_log), the model-angle sin / cos (dm_sincos) and
the first-octant atan (atan_ratio), against long double references.  Their
device twins are compared bitwise with these in tests/test_gpu_parity.py."""
import numpy as np

from pygcransac import _native as N

LD = np.longdouble


def _ulp_err(got, ref):
    ref64 = ref.astype(np.float64)
    ulp = np.spacing(np.abs(ref64))
    return np.abs(got.astype(LD) - ref) / ulp.astype(LD)


def _host(op, a, b=None):
    b = np.zeros_like(a) if b is None else b
    return np.array([N.lib.gcr_host_math(op, float(x), float(y)) for x, y in zip(a, b)])


def test_table_log_accuracy():
    rng = np.random.default_rng(1)
    x = np.concatenate([np.exp(rng.uniform(-700, 700, 20000)), rng.uniform(0.5, 1.5, 20000),
                        1.0 + rng.uniform(-1e-3, 1e-3, 20000), 1.0 + rng.uniform(-1e-12, 1e-12, 2000),
                        rng.uniform(1e-320, 1e-308, 500)])
    got = _host(0, x)
    err = _ulp_err(got, np.log(x.astype(LD)))
    assert float(err.max()) < 1.8                       # detmath.h: measured max 1.72 ulp
    assert N.lib.gcr_host_math(0, 1.0, 0.0) == 0.0      # c = 1 around 1
    specials = [0.0, -0.0, -1.0, np.inf, -np.inf, np.nan]
    out = _host(0, np.array(specials))
    assert out[0] == -np.inf and out[1] == -np.inf and np.isnan(out[2]) and out[3] == np.inf
    assert np.isnan(out[4]) and np.isnan(out[5])


def test_sincos_accuracy():
    rng = np.random.default_rng(2)
    x = np.concatenate([rng.uniform(-16, 16, 30000), rng.uniform(0, 2 * np.pi, 10000),
                        np.arange(-10, 11) * (np.pi / 2), [0.0, -0.0, 1e-300]])
    s, c = _host(9, x), _host(10, x)
    xl = x.astype(LD)
    rs, rc = np.sin(xl), np.cos(xl)
    # absolute error in units of ulp(1) (near the zeros relative error is
    # meaningless for a rotation) and relative error away from them
    assert float(np.max(np.abs(s.astype(LD) - rs))) < 2.3e-16
    assert float(np.max(np.abs(c.astype(LD) - rc))) < 2.3e-16
    big = np.abs(rs) > 1e-3
    assert float(_ulp_err(s[big], rs[big]).max()) < 1.5
    big = np.abs(rc) > 1e-3
    assert float(_ulp_err(c[big], rc[big]).max()) < 1.5
    assert N.lib.gcr_host_math(9, 0.0, 0.0) == 0.0 and N.lib.gcr_host_math(10, 0.0, 0.0) == 1.0
    assert np.isnan(N.lib.gcr_host_math(9, np.nan, 0.0)) and np.isnan(N.lib.gcr_host_math(10, np.inf, 0.0))


def test_atan_ratio_accuracy():
    rng = np.random.default_rng(3)
    d = 10.0 ** rng.uniform(-300, 300, 30000)
    n = d * rng.uniform(0, 1, 30000)
    got = _host(11, n, d)
    ref = np.arctan(n.astype(LD) / d.astype(LD))
    ok = ref > 0
    assert float(_ulp_err(got[ok], ref[ok]).max()) < 2.0
    assert N.lib.gcr_host_math(11, 0.0, 1.0) == 0.0
    assert abs(N.lib.gcr_host_math(11, 1.0, 1.0) - np.pi / 4) <= np.spacing(np.pi / 4)
