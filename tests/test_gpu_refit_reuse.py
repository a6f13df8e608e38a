"""Reuse of scoring launches.  The final refit reuses the adopted LO winner's score, raw counts and
inlier lists from its own scoring launch when the LO lists used the MSAC
threshold itself (two-class problems: Tlo = (1.5 thr)^2 and Tm = (2.25 thr)
thr rounding alike, rule 0), instead of rescoring it (GCRANSAC.h:628-675).
Runs must be identical with and without the reuse (GCR_LO_REUSE=0), and
equal to the oracle (covered by the golden and end-to-end tests)."""
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
