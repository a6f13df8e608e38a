"""Value sequences for the exact wave-parallel fold tests (k_lo_chain's
fold_exact_split): the reference adds MSAC terms one by one in fp64
(MSAC_scoring_function.hpp:53-107), so every case is checked against the
sequential left-to-right sum (np.add.accumulate)."""
import numpy as np


def sequential(v):
    s = 0.0
    for x in v:
        s = s + float(x)
    return s


def cases():
    rng = np.random.default_rng(7)
    out = {}
    # MSAC-like: -r^2 of inliers, r^2 uniform below a threshold
    out["msac"] = -rng.uniform(0, 2.25, 5000)
    out["msac_small_thr"] = -rng.uniform(0, 1e-6, 7000)
    # log-uniform magnitudes over 40 binades
    out["loguniform"] = -(10.0 ** rng.uniform(-20, 20, 4000))
    # ties: multiples of 2^-53 after -1.0 (ulp of [1, 2) is 2^-52: every odd
    # multiple of 2^-53 is an exact tie)
    t = -(rng.integers(1, 64, 3000).astype(np.float64)) * 2.0 ** -53
    out["ties"] = np.concatenate([[-1.0], t])
    # ties at every scale: k * ulp(s) / 2 relative to the running sum
    v = [-1.0]
    s = -1.0
    for _ in range(3000):
        u = np.spacing(abs(s))
        x = -float(rng.integers(0, 8)) * u / 2.0
        v.append(x)
        s = s + x
    out["ties_tracking"] = np.array(v)
    # binade crossings: values comparable to the sum
    out["crossings"] = -(2.0 ** rng.integers(-3, 3, 2000)) * (1.0 + rng.random(2000))
    # zeros, negative zeros, mixed
    z = -rng.uniform(0, 1, 3000)
    z[::3] = 0.0
    z[1::7] = -0.0
    out["zeros"] = z
    out["neg_zero_first"] = np.concatenate([[-0.0, -0.0, 0.0], -rng.uniform(0, 1, 500)])
    # subnormal start, then growing
    out["subnormal"] = np.concatenate([-np.full(100, 5e-324), -(10.0 ** rng.uniform(-320, -300, 500)),
                                       -rng.uniform(0, 1, 500)])
    # mixed signs (general case: the sum may shrink to a lower binade)
    out["mixed_signs"] = rng.normal(0, 1, 4000) * 10.0 ** rng.uniform(-3, 3, 4000)
    # huge, then tiny values (t >= 2^53 lanes)
    out["huge"] = np.concatenate([-rng.uniform(1e290, 1e300, 50), -rng.uniform(0, 1, 500),
                                  -rng.uniform(1e300, 1e307, 5)])
    # infinities and NaN
    inf = -rng.uniform(0, 1, 300)
    inf[150] = -np.inf
    out["inf"] = inf
    nan = -rng.uniform(0, 1, 300)
    nan[100] = np.nan
    out["nan"] = nan
    # lengths around the batch size
    for n in (2, 63, 64, 65, 127, 128, 129):
        out[f"len{n}"] = -rng.uniform(0, 3, n)
    return out
