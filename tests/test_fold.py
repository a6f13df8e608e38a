"""The block-parallel exact fold (kernels.hip fold_exact_block, used by
the small scorer) restated in numpy, chunk for chunk: a
128-value head added one by one (none for a chain that continues another),
chunks of 4, 8 or 16 values whose integer increments
rint(v / ulp) are summed exactly per run of one binade, runs separated by the
special values (predicted binade crossings, ties) that the walk adds on their
own; the walk folds value by value wherever a check fails.  Checked against
the sequential fp64 sum the reference computes (MSAC_scoring_function.hpp:
53-107) on adversarial sequences; the device kernel itself is checked against
the same sequences in tests/test_gpu_fold.py.  (Round 3's segment fold and
round 4's first split fold were replaced by this one; git history.)"""
import math

import numpy as np
import pytest

from fold_cases import cases, sequential


def _fold_seq(v, s):
    for x in v:
        s = s + float(x)
    return s


def _exp(x):
    return (int(np.float64(x).view(np.uint64)) >> 52) & 0x7ff


# --------------------------------------------------------- round 4: block ----
# fold_exact_block (kernels.hip): the in-order sum by all 1024 threads of a
# workgroup.  The first `head` values are added one by one (the sum is still
# small there); thread t then takes the t-th of the contiguous chunks of 4, 8
# or 16 values (the fewest threads the length needs) of the rest.  A block scan of approximate chunk sums gives every chunk an
# approximate start; walking its chunk with an approximate running sum, a
# thread adds the integer increments rint(v / U) (U the ulp of the binade the
# running sum is predicted to be in) and marks as special every value whose
# addition is predicted to leave the binade, and every tie.  Specials are
# numbered in sequence order (a block scan of the per-thread counts); the
# parts between consecutive specials are runs: run r's integer increments are
# summed over all threads (exact: integers of one sign below 2^53), its binade
# recorded.  One wave then walks the runs: s + U * A_r in one exact addition
# when the exact running sum lies in run r's binade and the result stays in it,
# then special r by an ordinary addition; the first failed check folds the rest
# value by value.  Any positive, NaN or too large value, a run whose parts
# disagree on the binade, more than BLK_SPECIALS specials or more than two in
# one chunk fold the whole sequence value by value.
BLK_THREADS = 1024
BLK_HEAD = 128
BLK_SPECIALS = 63
BLK_MAXM = 16          # values per chunk held in registers (longer ranges: one by one)


def _ulp_scale(be):
    return math.ldexp(1.0, 1075 - be)


def fold_exact_block(v, run=0.0, stats=None, head_len=BLK_HEAD, approx_start=None):
    """head_len = 0: a continuing chain (fold_exact_chains from >= 0), whose
    walk starts at the exact start itself.  approx_start: the chunks'
    approximate start in place of run (a continuing chain's is the chain it
    continues's approximate total)."""
    v = np.asarray(v, dtype=np.float64)
    n = v.size
    st = {"runs": 0, "specials": 0, "fallback": None}
    if n < head_len + BLK_THREADS // 4 or n - head_len > BLK_MAXM * BLK_THREADS:
        return _fold_seq(v, run)
    head = _fold_seq(v[:head_len], run)                   # exact (thread 64 c)
    # the chunks' approximate start: the device sums the head in any order
    # (a wave scan); the exact result does not depend on it
    ahead = float((run if approx_start is None else approx_start) + np.sum(v[:head_len]))
    rest = n - head_len
    mneed = (rest + BLK_THREADS - 1) // BLK_THREADS
    m = 4 if mneed <= 4 else (8 if mneed <= 8 else BLK_MAXM)
    bounds = [(head_len + min(rest, t * m), head_len + min(rest, t * m + m)) for t in range(BLK_THREADS)]
    with np.errstate(over="ignore", invalid="ignore"):
        a = np.array([_fold_seq(v[b:e], 0.0) for b, e in bounds])
        X = np.concatenate([[0.0], np.cumsum(a)[:-1]])    # exclusive scan (any order: approximate)
        parts, specials, bad = [], [], False
        for t, (b, e) in enumerate(bounds):
            P = ahead + X[t]
            acc = 0.0
            loc = []
            be = _exp(P)
            for j in range(b, e):
                x = float(v[j])
                be = _exp(P)
                if not (P < 0.0) or be < 53 or be >= 0x7fe:
                    bad = True
                    break
                t_ = x * _ulp_scale(be)
                r = float(np.rint(t_))
                if not (x <= 0.0) or not (abs(t_) < 2.0 ** 53):
                    bad = True
                    break
                Pn = P + x
                if abs(t_ - r) == 0.5 or _exp(Pn) != be:
                    loc.append((acc, be, j, x))
                    acc = 0.0
                else:
                    acc = acc + r
                P = Pn
            if bad:
                break
            if len(loc) > 2:
                bad = True
                break
            # parts: before special 1, between, after the last (binade of each)
            pb = [(p[0], p[1]) for p in loc] + [(acc, _exp(P) if loc else be)]
            parts.append(pb)
            specials.extend((j, x) for (_, _, j, x) in loc)
        if bad or len(specials) > BLK_SPECIALS:
            st["fallback"] = "all"
            if stats is not None:
                stats.update(st)
            return _fold_seq(v, run)
        nr = len(specials) + 1
        runA = [0.0] * nr
        runE = [set() for _ in range(nr)]
        rid = 0
        for pb in parts:
            for q, (A, e) in enumerate(pb):
                runA[rid] += A
                if not (A == 0.0 and q == len(pb) - 1 and False):
                    runE[rid].add(e)
                if q < len(pb) - 1:
                    rid += 1
    s = head
    pos = head_len
    for r in range(nr):
        E = runE[r]
        ok = len(E) == 1
        if ok:
            el = next(iter(E))
            ok = _exp(s) == el and s < 0.0
        if ok:
            S = s * _ulp_scale(el) + runA[r]
            ok = S > -2.0 ** 53
        if not ok:
            st["fallback"] = r
            s = _fold_seq(v[pos:], s)
            break
        s = S * math.ldexp(1.0, el - 1075)
        st["runs"] += 1
        if r < nr - 1:
            j, x = specials[r]
            s = s + x
            st["specials"] += 1
            pos = j + 1
    if stats is not None:
        stats.update(st)
    return s


@pytest.mark.parametrize("name", sorted(cases()))
def test_block_fold_restatement_equals_sequential_sum(name):
    v = cases()[name]
    for run in (0.0, -3.0, float(sequential(v[: len(v) // 3]))):
        for head_len in (BLK_HEAD, 0):
            got = fold_exact_block(v, run, head_len=head_len)
            ref = _fold_seq(v, run)
            assert np.float64(got).tobytes() == np.float64(ref).tobytes() or (ref != ref and got != got), (got, ref)


def test_block_fold_restatement_random():
    rng = np.random.default_rng(14)
    for _ in range(60):
        n = int(rng.integers(1, 9000))
        scale = 10.0 ** rng.uniform(-8, 8)
        v = -rng.uniform(0, scale, n)
        if rng.random() < 0.5:
            v = np.round(v / scale * 64) * scale / 64
        run = 0.0 if rng.random() < 0.5 else -float(rng.uniform(0, scale * n))
        assert np.float64(fold_exact_block(v, run)).tobytes() == np.float64(_fold_seq(v, run)).tobytes()


def test_block_fold_fast_on_msac_sums():
    """MSAC-like sums (LO trial scores): no fallback, one run per binade the
    sum passes through plus the tie-free crossings."""
    rng = np.random.default_rng(15)
    for n, run in ((5000, 0.0), (2500, 0.0), (2500, -1400.0), (8000, 0.0), (16000, 0.0)):
        v = -rng.uniform(0, 2.25, n)
        st = {}
        got = fold_exact_block(v, run, st)
        assert np.float64(got).tobytes() == np.float64(_fold_seq(v, run)).tobytes()
        assert st["fallback"] is None, st
        assert st["runs"] <= 24, st


def test_continuing_chain_exact_with_approximate_start():
    """The two-class fold's third chain (class 1 continuing the class-0 sum)
    starts its chunks from the class-0 chain's APPROXIMATE total: whatever the
    error of that start, the walk from the exact class-0 sum gives the
    sequential sum bit for bit (a wrong binade prediction only costs runs)."""
    rng = np.random.default_rng(16)
    for _ in range(40):
        n0, n1 = int(rng.integers(300, 6000)), int(rng.integers(300, 6000))
        v0 = -rng.uniform(0, 2.25, n0) * 10.0 ** rng.uniform(-6, 1)
        v1 = -rng.uniform(0, 2.25, n1) * 10.0 ** rng.uniform(-6, 1)
        a = _fold_seq(v0, 0.0)
        want = _fold_seq(v1, a)
        for err in (0.0, 1e-15, 1e-9, 1e-3, 0.5):
            st = {}
            got = fold_exact_block(v1, a, st, head_len=0, approx_start=a * (1.0 + err))
            assert np.float64(got).tobytes() == np.float64(want).tobytes(), (err, got, want)
