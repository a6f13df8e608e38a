"""The segment-parallel exact fold (kernels.hip fold_exact_seg, used by
k_lo_chain under GCR_LO_FOLD=wide) restated in numpy, segment for segment:
64 contiguous segments; approximate segment sums and a DPP-order scan give
each segment a binade; each segment adds rint(v / ulp) in four integer
accumulators and flags ties (fraction exactly 0.5), positive and too large
values; an in-order walk adds each valid segment in one exact fp64 addition
and folds the others value by value.  Checked against the sequential fp64
sum the reference computes (MSAC_scoring_function.hpp:53-107) on adversarial
sequences; the device kernel itself is checked against the same sequences in
tests/test_gpu_fold.py."""
import math

import numpy as np
import pytest

from fold_cases import cases, sequential


def _scan(x):
    """wave_incl_scan_f64's DPP order: row shifts 1, 2, 4, 8, then the row
    broadcasts of lanes 15 (into rows 1, 3) and 31 (into rows 2, 3)."""
    x = np.asarray(x, dtype=np.float64).copy()
    lanes = np.arange(64)
    for n in (1, 2, 4, 8):
        moved = np.zeros(64)
        ok = (lanes % 16) >= n
        moved[ok] = x[lanes[ok] - n]
        x = x + moved
    moved = np.zeros(64)
    moved[16:32] = x[15]
    moved[48:64] = x[47]
    x = x + moved
    moved = np.zeros(64)
    moved[32:64] = x[31]
    return x + moved


def _fold_seq(v, s):
    for x in v:
        s = s + float(x)
    return s


def _exp(x):
    return (int(np.float64(x).view(np.uint64)) >> 52) & 0x7ff


def fold_exact_seg(v, run=0.0):
    """kernels.hip fold_exact_seg, segment for segment."""
    v = np.asarray(v, dtype=np.float64)
    n = v.size
    if n < 512:
        return _fold_seq(v, run)
    L = ((n + 63) // 64) | 1
    a, I, E = np.zeros(64), np.zeros(64), np.zeros(64, dtype=np.int64)
    flag = np.zeros(64, dtype=bool)
    with np.errstate(over="ignore", invalid="ignore"):
        for lane in range(64):
            seg = v[min(n, lane * L):min(n, lane * L + L)]
            acc = np.zeros(4)
            m = seg.size - seg.size % 4
            for q in range(0, m, 4):
                acc = acc + seg[q:q + 4]
            acc[0] = _fold_seq(seg[m:], acc[0])
            a[lane] = (acc[0] + acc[1]) + (acc[2] + acc[3])
        X = _scan(a)
        for lane in range(64):
            seg = v[min(n, lane * L):min(n, lane * L + L)]
            g = run + (X[lane] - a[lane])
            be, be2 = _exp(g), _exp(g + a[lane])
            f = not (g < 0.0) or be < 53 or be == 0x7ff or be2 != be
            iU = math.ldexp(1.0, 1075 - (1075 if f else be))
            t = seg * iU
            r = np.rint(t)
            bad = bool(np.any(seg > 0.0) or np.any(~(np.abs(t) < 2.0 ** 53)) or np.any(np.abs(t - r) == 0.5))
            acc = np.zeros(4)
            m = seg.size - seg.size % 4
            for q in range(0, m, 4):
                acc = acc + r[q:q + 4]
            acc[0] = _fold_seq(r[m:], acc[0])
            f = f or bad
            flag[lane] = f
            I[lane] = 0.0 if f else (acc[0] + acc[1]) + (acc[2] + acc[3])
            E[lane] = 0 if f else be
    s = run
    for lane in range(64):
        seg = v[min(n, lane * L):min(n, lane * L + L)]
        if seg.size == 0:
            break
        el = int(E[lane])
        if el != 0 and _exp(s) == el and s < 0.0:
            S = s * math.ldexp(1.0, 1075 - el) + I[lane]
            if -2.0 ** 53 < S <= -2.0 ** 52:
                s = S * math.ldexp(1.0, el - 1075)
                continue
        s = _fold_seq(seg, s)
    return s


@pytest.mark.parametrize("name", sorted(cases()))
def test_fold_restatement_equals_sequential_sum(name):
    v = cases()[name]
    got = fold_exact_seg(v)
    ref = sequential(v)
    assert np.float64(got).tobytes() == np.float64(ref).tobytes() or (ref != ref and got != got), (got, ref)


def test_fold_restatement_random_prefixes():
    rng = np.random.default_rng(11)
    for _ in range(200):
        n = int(rng.integers(1, 3000))
        scale = 10.0 ** rng.uniform(-8, 8)
        v = -rng.uniform(0, scale, n)
        if rng.random() < 0.5:                       # quantised values: frequent ties
            v = np.round(v / scale * 64) * scale / 64
        assert np.float64(fold_exact_seg(v)).tobytes() == np.float64(sequential(v)).tobytes()
