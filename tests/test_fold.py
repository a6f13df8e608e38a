"""The segment-parallel exact fold (kernels.hip fold_exact_split, used by
k_lo_chain under GCR_LO_FOLD=wide) restated in numpy, segment for segment:
a 16-value first segment and 63 equal ones; approximate segment sums and a
DPP-order scan give each segment a binade; each segment adds rint(v / ulp)
as exact integers in parts separated by up to two special values (binade
crossings, ties); an in-order walk adds each part in one exact fp64 addition
and each special value on its own, and folds value by value wherever a check
fails.  Checked against the sequential fp64 sum the reference computes
(MSAC_scoring_function.hpp:53-107) on adversarial sequences; the device
kernel itself is checked against the same sequences in
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


# ------------------------------------------------------------------ round 4 --
# fold_exact_split (kernels.hip): the segment fold with up to two "special"
# values per segment handled exactly -- a binade crossing (predicted from the
# approximate start) or a tie (a value whose increment ends in exactly .5 ulp,
# where round-to-even depends on the running sum's parity).  A short first
# segment (16 values, usually folded value by value from the chain's start),
# 63 segments after it.  Phase 2 adds the integer increments at the
# segment's ulp U in parts separated by the specials (2U after a crossing);
# the walk applies each part in one exact addition and each special by an
# ordinary addition, each verified against the exact running sum; a failed
# check, or a third special, folds the rest of the segment value by value.
L0_SPLIT = 16
MAX_SPECIAL = 2


def _seg_bounds(n, lane):
    L = ((n - L0_SPLIT + 62) // 63) | 1
    if lane == 0:
        return 0, min(n, L0_SPLIT)
    b = min(n, L0_SPLIT + (lane - 1) * L)
    return b, min(n, b + L)


def _ldexp(e):
    return math.ldexp(1.0, e)


def _phase2(seg, g, be, flag):
    """One lane's records: parts A[0..k], specials (index, value, crossing?),
    tail index (-1: none), validity."""
    bs = 1075 if flag else be
    iU = _ldexp(1075 - bs)
    P = g * iU
    mode = 0
    acc = 0.0
    A, SPI, SPV, SPX = [], [], [], []
    tail = -1
    bad = False
    for j, x in enumerate(seg):
        x = float(x)
        t = x * (iU * 0.5 ** mode)
        r = float(np.rint(t))
        if not (x <= 0.0) or not (abs(t) < 2.0 ** 53):
            bad = True
        tie = abs(t - r) == 0.5
        cross = P + r <= -2.0 ** 53
        if tie or cross:
            if len(SPI) == MAX_SPECIAL:
                tail = j
                break
            A.append(acc)
            acc = 0.0
            SPI.append(j)
            SPV.append(x)
            SPX.append(cross)
            if cross:
                mode += 1
                P = (P + r) * 0.5
            else:
                P = P + r
            continue
        P = P + r
        acc = acc + r
    A.append(acc)
    return A, SPI, SPV, SPX, tail, not (flag or bad)


def fold_exact_split(v, run=0.0, stats=None):
    """kernels.hip fold_exact_split, segment for segment (stats: counts of
    the walk's paths: "fast" whole segments, "slow" value by value from the
    segment start, "tail" value by value from a later point)."""
    st = {"fast": 0, "tail": 0, "slow": 0, "specials": 0}
    v = np.asarray(v, dtype=np.float64)
    n = v.size
    if n < 512:
        return _fold_seq(v, run)
    a = np.zeros(64)
    rec = []
    with np.errstate(over="ignore", invalid="ignore"):
        for lane in range(64):
            b, e = _seg_bounds(n, lane)
            seg = v[b:e]
            acc = np.zeros(4)
            m = seg.size - seg.size % 4
            for q in range(0, m, 4):
                acc = acc + seg[q:q + 4]
            acc[0] = _fold_seq(seg[m:], acc[0])
            a[lane] = (acc[0] + acc[1]) + (acc[2] + acc[3])
        X = _scan(a)
        for lane in range(64):
            b, e = _seg_bounds(n, lane)
            g = run + (X[lane] - a[lane])
            be, bend = _exp(g), _exp(g + a[lane])
            flag = not (g < 0.0) or be < 53 or be >= 0x7fd or bend > be + MAX_SPECIAL
            rec.append((be,) + _phase2(v[b:e], g, be, flag))
    s = run
    for lane in range(64):
        b, e = _seg_bounds(n, lane)
        if b >= e:
            break
        be, A, SPI, SPV, SPX, tail, ok = rec[lane]
        if not ok:
            s = _fold_seq(v[b:e], s)
            st["slow"] += 1
            continue
        el = be
        pos = b                       # first value not yet added
        done = False
        for q in range(len(A)):
            if not (_exp(s) == el and s < 0.0):
                break
            S = s * _ldexp(1075 - el) + A[q]
            if not (S > -2.0 ** 53):
                break
            s = S * _ldexp(el - 1075)
            if q == len(SPI):
                pos = e if tail < 0 else b + tail
                done = True
                break
            s = s + SPV[q]
            st["specials"] += 1
            pos = b + SPI[q] + 1
            if SPX[q]:
                el = el + 1
        if done and pos == e:
            st["fast"] += 1
            continue
        st["slow" if pos == b else "tail"] += 1
        s = _fold_seq(v[pos:e], s)
    if stats is not None:
        stats.update(st)
    return s


@pytest.mark.parametrize("name", sorted(cases()))
def test_split_fold_restatement_equals_sequential_sum(name):
    v = cases()[name]
    for run in (0.0, -3.0, float(sequential(v[: len(v) // 3]))):
        got = fold_exact_split(v, run)
        ref = _fold_seq(v, run)
        assert np.float64(got).tobytes() == np.float64(ref).tobytes() or (ref != ref and got != got), (got, ref)


def test_split_fold_restatement_random_prefixes():
    rng = np.random.default_rng(12)
    for _ in range(120):
        n = int(rng.integers(1, 3000))
        scale = 10.0 ** rng.uniform(-8, 8)
        v = -rng.uniform(0, scale, n)
        if rng.random() < 0.5:                       # quantised values: frequent ties
            v = np.round(v / scale * 64) * scale / 64
        run = 0.0 if rng.random() < 0.5 else -float(rng.uniform(0, scale * n))
        assert np.float64(fold_exact_split(v, run)).tobytes() == np.float64(_fold_seq(v, run)).tobytes()


def test_split_fold_fast_paths_dominate_msac_sums():
    """On MSAC-like sums (the LO trial scores, 2500-5000 inliers) every
    segment but the first takes an exact fast path, the ones crossing a
    binade or holding a tie included (those values added on their own)."""
    rng = np.random.default_rng(13)
    for n, run in ((5000, 0.0), (2500, 0.0), (2500, -1400.0)):
        v = -rng.uniform(0, 2.25, n)
        st = {}
        got = fold_exact_split(v, run, st)
        assert np.float64(got).tobytes() == np.float64(_fold_seq(v, run)).tobytes()
        assert st["slow"] <= 1 and st["tail"] <= 1 and st["specials"] >= 1, st
