"""The wave-parallel exact fold (kernels.hip fold_exact_wave, used by
k_lo_chain) restated in numpy, lane for lane: 256 values per step, four
consecutive ones per lane, each scaled by 1 / ulp(s) and rounded to an
integer; the lane's in-order partial sums, an inclusive scan of the lane
totals on s / ulp(s) in the kernel's DPP order; the first value that ties
(fraction exactly 0.5), is positive, too large or leaves the binade is added
by one ordinary fp64 addition.  Checked against the sequential fp64 sum the
reference computes (MSAC_scoring_function.hpp:53-107) on adversarial
sequences; the device kernel itself is checked against the same sequences in
tests/test_gpu_fold.py."""
import math

import numpy as np
import pytest

from fold_cases import cases, sequential


def _dpp(x, ctrl):
    """DPP moves of wave_incl_scan_f64 (0 where nothing moves in)."""
    out = np.zeros(64)
    lanes = np.arange(64)
    if ctrl[0] == "shr":                         # row_shr:n inside rows of 16
        n = ctrl[1]
        src = lanes - n
        ok = (lanes % 16) >= n
        out[ok] = x[src[ok]]
    elif ctrl[0] == "bcast15":                   # lane 15 of the row before, into rows 1 and 3
        for r in (1, 3):
            out[16 * r:16 * r + 16] = x[16 * r - 1]
    elif ctrl[0] == "bcast31":                   # lane 31 into rows 2 and 3
        out[32:64] = x[31]
    elif ctrl[0] == "wshr1":                     # wave_shr:1
        out[1:] = x[:-1]
    return out


def _scan(x):
    for c in (("shr", 1), ("shr", 2), ("shr", 4), ("shr", 8), ("bcast15",), ("bcast31",)):
        x = x + _dpp(x, c)
    return x


def fold_exact_wave(v, run=0.0, per=4):
    """kernels.hip fold_exact_wave, lane for lane (64 lanes x `per` values)."""
    v = np.asarray(v, dtype=np.float64)
    k, e = 0, v.size
    lanes = np.arange(64)
    while k < e:
        n = min(64 * per, e - k)
        be = (int(np.float64(run).view(np.uint64)) >> 52) & 0x7ff
        if be < 53 or be == 0x7ff or not run < 0.0:
            run = run + float(v[k])
            k += 1
            continue
        U = math.ldexp(1.0, be - 1075)
        iU = math.ldexp(1.0, 1075 - be)
        pos = lanes[:, None] * per + np.arange(per)[None, :]
        x0 = np.zeros((64, per))
        x0[pos < n] = v[k:k + n]
        with np.errstate(over="ignore", invalid="ignore"):
            t = x0 * iU
            ni = np.rint(t)
            ok = ~(x0 > 0.0) & (np.abs(t) < 2.0 ** 53) & (np.abs(t - ni) != 0.5)
            pre = np.zeros((64, per))
            acc = np.zeros(64)
            for j in range(per):                     # in-lane order
                acc = acc + ni[:, j]
                pre[:, j] = acc
            S0 = run * iU
            X = _scan(np.where(lanes == 0, S0 + acc, acc))
            B = np.where(lanes == 0, S0, _dpp(X, ("wshr1",)))
            q = B[:, None] + pre
            good = (ok & (q > -2.0 ** 53) & (q <= -2.0 ** 52)) | (pos >= n)
        badpos = np.nonzero(~good.reshape(-1))[0]
        f = min(n, int(badpos[0])) if badpos.size else n
        if f > 0:
            g = f - 1
            run = float(q[g // per, g % per]) * U
        if f < n:
            run = run + float(v[k + f])
            k += f + 1
        else:
            k += n
    return run


@pytest.mark.parametrize("name", sorted(cases()))
def test_fold_restatement_equals_sequential_sum(name):
    v = cases()[name]
    got = fold_exact_wave(v)
    ref = sequential(v)
    assert np.float64(got).tobytes() == np.float64(ref).tobytes() or (ref != ref and got != got), (got, ref)


def test_fold_restatement_random_prefixes():
    rng = np.random.default_rng(11)
    for _ in range(200):
        n = int(rng.integers(1, 700))
        scale = 10.0 ** rng.uniform(-8, 8)
        v = -rng.uniform(0, scale, n)
        if rng.random() < 0.5:                       # quantised values: frequent ties
            v = np.round(v / scale * 64) * scale / 64
        assert np.float64(fold_exact_wave(v)).tobytes() == np.float64(sequential(v)).tobytes()
