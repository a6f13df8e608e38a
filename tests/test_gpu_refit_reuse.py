"""Reuse of scoring launches.  The final refit reuses the adopted LO winner's
score, raw counts and MSAC inlier lists from its own small-scorer launch
(which scored it with the MSAC threshold and mirrored its MSAC ballots),
instead of rescoring it (GCRANSAC.h:628-675) -- for every estimator, unless
one of the winner's MSAC decisions was flagged for the glibc recheck.  Runs
must be identical with and without the reuse (GCR_LO_REUSE=0), the check mode
(GCR_LO_CACHE_CHECK=1) rescores and requires bit-identical score, counts and
lists, and runs equal the oracle (the golden and end-to-end tests)."""
import numpy as np
import pytest

import pygcransac
from gcr_testutil import bits
from pygcransac import synthetic as S

pytestmark = pytest.mark.gpu


def _run(fs, fo, ts, to, seed, conf):
    H, sm, om, model, st = pygcransac.findRectifyingHomographySIFT(fs, fo, ts, to, 0.0, 0, 10**6, 50, seed=seed,
                                                                  confidence=conf, return_stats=True)
    return (None if H is None else bits(H).tobytes(), sm.tobytes(), om.tobytes(),
            st["iteration_number"], st["local_optimization_number"], st["graph_cut_number"],
            bits(st["score"]).tobytes())


@pytest.mark.parametrize("n,seed,conf", [(5000, 100, 0.99), (5000, 103, 0.99), (2000, 7, 0.999), (1200, 11, 0.95)])
def test_refit_reuse_equals_rescore(n, seed, conf, monkeypatch):
    fs, fo, _, _, ts, to = S.problem_m2(n, n, seed=seed)
    a = _run(fs, fo, ts, to, seed, conf)
    monkeypatch.setenv("GCR_LO_REUSE", "0")
    b = _run(fs, fo, ts, to, seed, conf)
    assert a == b
    assert a[0] is not None and a[4] > 0
    monkeypatch.setenv("GCR_LO_REUSE", "1")
    monkeypatch.setenv("GCR_LO_CACHE_CHECK", "1")
    assert _run(fs, fo, ts, to, seed, conf) == a


@pytest.mark.parametrize("kind", ["m1", "h", "f"])
def test_refit_reuse_check_mode_other_estimators(kind, monkeypatch):
    # the cache is used by every estimator: the check mode's rescore agrees
    monkeypatch.setenv("GCR_LO_CACHE_CHECK", "1")
    if kind == "m1":
        f, _, thr = S.problem_m1(4000, seed=21)
        out = pygcransac.findRectifyingHomographyScaleOnly(f, thr, 0.0, 0, 10**6, 50, seed=3, confidence=0.99)
    elif kind == "h":
        c, _, _, thr = S.problem_h(3000, 0.5, seed=22)
        out = pygcransac.findHomography(c, 960, 1280, 960, 1280, threshold=thr, conf=0.99, seed=3)
    else:
        c, _, _, thr = S.problem_f(3000, 0.6, seed=23)
        out = pygcransac.findFundamentalMatrix(c, 960, 1280, 960, 1280, threshold=thr, conf=0.99, seed=3)
    assert out[0] is not None


@pytest.mark.parametrize("budget", ["fixed", "adaptive", "tiny", "floor"])
def test_chunk_list_bits_equal_mask_launches(budget, monkeypatch):
    # small-scored chunks write every slot's LO lists into pinned memory and
    # the LO of a new best from such a chunk starts from them instead of a
    # mask launch (GCR_CHUNK_LISTS=0): identical runs for every estimator and
    # budget ("tiny": 37-slot chunks, the two buffer sets reused many times)
    from test_gpu_summary import SOLVERS, _run as run_problem

    for kind in SOLVERS:
        a = run_problem(kind, budget, monkeypatch, {})
        b = run_problem(kind, budget, monkeypatch, {"GCR_CHUNK_LISTS": "0"})
        assert a == b, kind


@pytest.mark.parametrize("budget", ["fixed", "adaptive", "tiny", "floor"])
def test_chunk_msac_bits_equal_mask_launches(budget, monkeypatch):
    # small-scored chunks also mirror every slot's MSAC ballots, and the final
    # refit of a run whose best is still the chunk hypothesis it was found as
    # takes its inlier lists from them (GCR_CHUNK_MSAC=0: mask launches):
    # identical runs for every estimator and budget
    from test_gpu_summary import SOLVERS, _run as run_problem

    for kind in SOLVERS:
        a = run_problem(kind, budget, monkeypatch, {})
        b = run_problem(kind, budget, monkeypatch, {"GCR_CHUNK_MSAC": "0"})
        assert a == b, kind


def test_chunk_msac_lists_used_at_the_bench_call():
    # bench.py's latency call (M2 5000 + 5000, seeds 100..110): over the
    # eleven seeds some runs end on a chunk-found best whose refit lists come
    # from the chunk's MSAC ballots (test_gpu_glibc.py checks those calls
    # against the oracle's GLIBC mode)
    fs, fo, _, _, ts, to = S.problem_m2(5000, 5000, seed=20251121)
    used = 0
    for seed in range(100, 111):
        out = pygcransac.findRectifyingHomographySIFT(fs, fo, ts, to, 0.0, 0, 10**7, 50, seed=seed,
                                                      confidence=0.99, return_stats=True)
        used += out[-1]["chunk_msac_lists"]
    assert used > 0
