#!/usr/bin/env python3
"""Frozen graph-cut tie fixtures (tests/golden/graphcut_ties.json).

Each case is a labeling() call (GCRANSAC.h:759-870) on a few points whose
energies tie on purpose: residuals exactly at the truncated threshold
(r2 == sqt, where both unary terms are 0), equal residuals, lambda chosen so
every term is a dyadic rational (all sums exact).  The expected SINK set is
derived independently of any BK code: the reference reads the labels with
what_segment(i) == SINK and default_segm = SOURCE (GCRANSAC.h:865,
graph.h:115-117, :480-488), so a node is SINK exactly when it can still reach
the sink in the residual graph of a maximum flow -- the minimal sink side,
which is the intersection of the sink sets of all minimum-energy labelings.
Here that intersection is taken over an exhaustive enumeration of the 2^n
labelings of the energy (unary and pairwise terms as labeling() adds them).

Written once; the test checks the product (graphcut.h) and the oracle's BK
restatement against these frozen expectations, never regenerating them.
"""
import itertools
import json
import os
import sys

import numpy as np


def energy_terms(r2, sqt, lam, edges):
    oml = 1.0 - lam
    q = np.clip(r2 / sqt, 0.0, 1.0)
    unary = np.zeros((r2.size, 2))
    inl = r2 <= sqt
    unary[inl, 0] = oml * (1.0 - q[inl])
    unary[~inl, 1] = oml * (1.0 - (1.0 - q[~inl]))
    pair = [(lam * 0.5 * (q[u] + q[v]), lam, lam, 0.0) for u, v in edges]
    return unary, pair


def minimal_sink_set(r2, sqt, lam, edges):
    unary, pair = energy_terms(np.asarray(r2, float), sqt, lam, edges)
    n = len(r2)
    best, sets = None, []
    for x in itertools.product((0, 1), repeat=n):
        e = sum(unary[i, x[i]] for i in range(n))
        e += sum(p[2 * x[u] + x[v]] for (u, v), p in zip(edges, pair))
        if best is None or e < best:
            best, sets = e, [x]
        elif e == best:
            sets.append(x)
    return [int(all(s[i] for s in sets)) for i in range(n)], len(sets)


def cell_edges(cells_of):
    """labeling()'s grid edges: every pair (i < j) sharing a cell, i ascending."""
    return [(i, j) for i in range(len(cells_of)) for j in range(i + 1, len(cells_of)) if cells_of[i] == cells_of[j]]


def main():
    sqt = 4.0
    cases = []
    # (name, r2 per point, cell of each point, lambda)
    specs = [
        ("one point at the threshold, alone", [sqt], [0], 0.5),
        ("two points at the threshold", [sqt, sqt], [0, 0], 0.5),
        ("threshold point + outlier: three optimal labelings", [sqt, 9.0], [0, 0], 0.5),
        ("threshold point + outlier, lambda 0.75", [sqt, 16.0], [0, 0], 0.75),
        ("threshold point + deep inlier", [sqt, 0.0], [0, 0], 0.5),
        ("three at the threshold + outlier", [sqt, sqt, sqt, 8.0], [0, 0, 0, 0], 0.5),
        ("half-threshold pair + outlier pair", [2.0, 2.0, 12.0, 12.0], [0, 0, 0, 0], 0.5),
        ("two cells, mixed", [sqt, 9.0, 1.0, sqt, sqt], [0, 0, 1, 1, 1], 0.75),
        ("lambda 1: pairwise terms only", [sqt, 1.0, 20.0], [0, 0, 0], 1.0),
        ("lambda 0.25, five at the threshold + one outlier", [sqt] * 5 + [5.0], [0] * 6, 0.25),
    ]
    # searched: small dyadic configurations with several optimal labelings
    rng = np.random.default_rng(2026)
    found = 0
    while found < 14:
        n = int(rng.integers(2, 7))
        r2 = [float(v) for v in rng.choice([0.0, 1.0, 2.0, sqt, sqt, sqt, 6.0, 8.0, 16.0], n)]
        cells_of = [int(v) for v in rng.integers(0, 2, n)]
        lam = float(rng.choice([0.125, 0.25, 0.5, 0.75]))
        sink, nopt = minimal_sink_set(r2, sqt, lam, cell_edges(cells_of))
        if nopt >= 2 and 0 < sum(sink) < n or (nopt >= 3 and found < 4):
            specs.append((f"searched tie {found}", r2, cells_of, lam))
            found += 1
    for name, r2, cells_of, lam in specs:
        edges = cell_edges(cells_of)
        sink, nopt = minimal_sink_set(r2, sqt, lam, edges)
        # points: cell c of an 8 x 8 grid of 10-px cells (4-D correspondences)
        pts = [[10.0 * c + 1.0 + 0.5 * k, 1.0, 10.0 * c + 1.0 + 0.5 * k, 1.0] for k, c in enumerate(cells_of)]
        cases.append({"name": name, "r2": r2, "sqt": sqt, "lambda": lam, "points": pts,
                      "cell_size": [10.0, 10.0, 10.0, 10.0], "cells": 8, "edges": edges,
                      "optimal_labelings": nopt, "sink": sink})
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "graphcut_ties.json")
    if os.path.exists(out) and "--force" not in sys.argv:
        sys.exit(f"{out} exists: the fixtures are frozen (pass --force to rewrite)")
    with open(out, "w") as f:
        json.dump({"generator": "tools/gen_gc_ties.py", "cases": cases}, f, indent=1)
    for c in cases:
        print(f"{c['name']:55s} optimal labelings {c['optimal_labelings']}  SINK {c['sink']}")


if __name__ == "__main__":
    main()
