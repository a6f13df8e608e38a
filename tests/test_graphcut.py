"""Graph-cut labeling (CPU): the neighbourhood grid's edge list, the BK
st-mincut and labeling() itself, product (graphcut.h through the C ABI host
hooks) against the oracle's restatement (oracle/gcr_oracle.cpp GridGraph /
BKGraph, following grid_neighborhood_graph.h:229-301, energy.h:204-245,
graph.h / maxflow.ti, GCRANSAC.h:759-870) and against independent checkers:
brute-force minimisation over every labeling of small energies, and scipy's
max-flow on integer-capacity graphs.

BK's labeling is SINK for exactly the nodes that can still reach the sink in
the residual graph of a maximum flow: the minimal sink side, the same for
every maximum flow, i.e. the intersection of the sink sets of all optimal
labelings."""
import ctypes as C
import itertools

import numpy as np
import pytest

import oracle_ffi as O
from pygcransac import _native as N
from pygcransac import synthetic as S

u32p = C.POINTER(C.c_uint32)
u8p = C.POINTER(C.c_uint8)
dp = C.POINTER(C.c_double)


def product_bk(unary, edges, pair):
    u = np.ascontiguousarray(np.asarray(unary, dtype=np.float64).reshape(-1, 2))
    e = np.ascontiguousarray(np.asarray(edges, dtype=np.uint32).reshape(-1, 2))
    pr = np.ascontiguousarray(np.asarray(pair, dtype=np.float64).reshape(-1, 4))
    seg = np.zeros(u.shape[0], dtype=np.uint8)
    N.check(N.lib.gcr_host_bk_energy(u.shape[0], u.ctypes.data_as(dp), e.ctypes.data_as(u32p),
                                     pr.ctypes.data_as(dp), e.shape[0], seg.ctypes.data_as(u8p)))
    return seg.astype(bool)


def product_edges(points, cell_size, cells):
    pts = np.ascontiguousarray(points, dtype=np.float64)
    cs = np.ascontiguousarray(cell_size, dtype=np.float64)
    m = C.c_size_t()
    N.check(N.lib.gcr_host_grid_edges(pts.ctypes.data_as(dp), pts.shape[0], pts.shape[1], cs.ctypes.data_as(dp),
                                      cells, None, 0, C.byref(m)))
    out = np.zeros((max(m.value, 1), 2), dtype=np.uint32)
    N.check(N.lib.gcr_host_grid_edges(pts.ctypes.data_as(dp), pts.shape[0], pts.shape[1], cs.ctypes.data_as(dp),
                                      cells, out.ctypes.data_as(u32p), m.value, C.byref(m)))
    return out[:m.value]


def product_labeling(r2, sqt, lam, points=None, cell_size=(0.0,) * 4, cells=0):
    """labeling() as the engine runs it: the grid built from `points`, every
    multi-point cell cut on its own (its own component of the graph)."""
    r = np.ascontiguousarray(r2, dtype=np.float64)
    seg = np.zeros(r.size, dtype=np.uint8)
    pts = np.ascontiguousarray(points if points is not None else np.zeros((r.size, 1)), dtype=np.float64)
    cs = np.ascontiguousarray(cell_size, dtype=np.float64)
    N.check(N.lib.gcr_host_labeling(r.ctypes.data_as(dp), r.size, sqt, lam, pts.ctypes.data_as(dp), pts.shape[1],
                                    cs.ctypes.data_as(dp), cells, seg.ctypes.data_as(u8p)))
    return seg.astype(bool)


def labeling_energy(r2, sqt, lam, edges):
    """labeling()'s energy terms (GCRANSAC.h:789-857) in the add_term form."""
    oml = 1.0 - lam
    q = np.clip(r2 / sqt, 0.0, 1.0)
    unary = np.zeros((r2.size, 2))
    inl = r2 <= sqt
    unary[inl, 0] = oml * (1.0 - q[inl])
    unary[~inl, 1] = oml * (1.0 - (1.0 - q[~inl]))
    e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
    e00 = 0.5 * (q[e[:, 0]] + q[e[:, 1]])
    pair = np.column_stack([e00 * lam, np.full(len(e), lam), np.full(len(e), lam), np.zeros(len(e))])
    return unary, pair


def energy_of(x, unary, edges, pair):
    x = np.asarray(x, dtype=np.int64)
    e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
    val = unary[np.arange(len(x)), x].sum()
    if len(e):
        val += pair[np.arange(len(e)), 2 * x[e[:, 0]] + x[e[:, 1]]].sum()
    return val


def random_submodular(rng, n, m):
    """Dyadic values (exact arithmetic) with A + D <= B + C on every edge; some
    edges exercise add_term2's B < 0 and C < 0 branches."""
    unary = rng.integers(0, 9, (n, 2)) / 4.0
    edges = []
    while len(edges) < m:
        u, v = rng.choice(n, 2, replace=False)
        edges.append((u, v))
    pair = np.zeros((m, 4))
    for k in range(m):
        A, D = rng.integers(0, 9, 2) / 4.0
        if rng.random() < 0.3:
            B = rng.integers(-4, 1) / 4.0                 # B < A possible -> add_term2's B < 0 branch
            C_ = A + D - B + rng.integers(0, 5) / 4.0
        else:
            B, C_ = rng.integers(0, 9, 2) / 4.0
            C_ = max(C_, A + D - B)
        pair[k] = (A, B, C_, D) if rng.random() < 0.5 else (A, C_, B, D)
    return unary, np.array(edges, dtype=np.uint32), pair


@pytest.mark.parametrize("seed", range(40))
def test_bk_equals_brute_force_minimal_sink_set(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 11))
    m = int(rng.integers(0, 2 * n + 1))
    unary, edges, pair = random_submodular(rng, n, m)
    energies = np.array([energy_of(x, unary, edges, pair) for x in itertools.product((0, 1), repeat=n)])
    best = energies.min()
    labelings = np.array(list(itertools.product((0, 1), repeat=n)), dtype=bool)
    optimal = labelings[energies == best]
    expect = np.logical_and.reduce(optimal, axis=0)      # the minimal sink side
    got = product_bk(unary, edges, pair)
    ref, _ = O.bk_energy(unary, edges, pair)
    assert np.array_equal(got, ref)
    assert energy_of(got.astype(int), unary, edges, pair) == best
    assert np.array_equal(got, expect)


def test_bk_matches_scipy_max_flow_on_integer_graphs():
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import maximum_flow

    rng = np.random.default_rng(7)
    for trial in range(6):
        n, m = 300, 1500
        # Potts-form pairwise terms of labeling() with integer weights
        unary = np.zeros((n, 2))
        side = rng.random(n) < 0.5
        unary[side, 0] = rng.integers(1, 40, side.sum())
        unary[~side, 1] = rng.integers(1, 40, (~side).sum())
        edges = set()
        while len(edges) < m:
            u, v = rng.choice(n, 2, replace=False)
            if (u, v) not in edges and (v, u) not in edges:
                edges.add((int(u), int(v)))
        edges = np.array(sorted(edges), dtype=np.uint32)
        lam = rng.integers(5, 30, m).astype(float)
        a = np.minimum(rng.integers(0, 30, m), lam)
        pair = np.column_stack([a, lam, lam, np.zeros(m)])
        got = product_bk(unary, edges, pair)
        assert np.array_equal(got, O.bk_energy(unary, edges, pair)[0])
        # the same energy as an st-graph (energy.h add_term2 decomposition):
        # node i: s -> i costs E_i(1), i -> t costs E_i(0) (+ A of its edges as x)
        s, t = n, n + 1
        cap = {}

        def add(i, j, c):
            if c > 0:
                cap[(i, j)] = cap.get((i, j), 0) + int(c)

        e0 = unary[:, 0].copy()
        for (x, y), (A, B, Cc, D) in zip(edges, pair):
            e0[x] += A                                    # add_tweights(x, D=0, A)
            add(x, y, B - A)
            add(y, x, Cc - D)
        for i in range(n):
            add(s, i, unary[i, 1])
            add(i, t, e0[i])
        rows, cols = zip(*cap.keys())
        G = csr_matrix((list(cap.values()), (rows, cols)), shape=(n + 2, n + 2), dtype=np.int32)
        res = maximum_flow(G, s, t)
        F = res.flow.toarray()
        Cm = G.toarray()
        resid = Cm - F                                     # includes reverse residuals (F antisymmetric)
        # nodes that can reach t in the residual graph = the minimal sink side
        reach = np.zeros(n + 2, dtype=bool)
        reach[t] = True
        stack = [t]
        while stack:
            v = stack.pop()
            for u in np.flatnonzero(resid[:, v] > 0):
                if not reach[u]:
                    reach[u] = True
                    stack.append(u)
        assert np.array_equal(got, reach[:n]), trial
        assert energy_of(got.astype(int), unary, edges, pair) == res.flow_value      # min cut = min energy


def test_grid_edges_match_oracle_including_collisions_and_non_finite():
    rng = np.random.default_rng(3)
    corr, _, _, _ = S.problem_h(3000, 0.5, seed=5)
    for cells, sizes in ((8, (1280 / 8, 960 / 8, 1280 / 8, 960 / 8)), (4, (400.0, 300.0, 400.0, 300.0)),
                         (3, (100.0, 100.0, 100.0, 100.0))):         # the last: indices beyond the grid collide
        got = product_edges(corr, sizes, cells)
        ref = O.grid_edges(corr, sizes, cells)
        assert np.array_equal(got, ref)
        assert len(got) > 0
    bad = corr[:400].copy()
    bad[::7, 0] = -35.5                                  # negative coordinates
    bad[::11, 1] = np.nan
    bad[::13, 2] = np.inf
    got = product_edges(bad, (160.0, 120.0, 160.0, 120.0), 8)
    assert np.array_equal(got, O.grid_edges(bad, (160.0, 120.0, 160.0, 120.0), 8))
    # labeling() order: first endpoint non-decreasing, each pair once, i < j
    assert np.all(np.diff(got[:, 0].astype(np.int64)) >= 0) and np.all(got[:, 0] < got[:, 1])
    assert len({(int(a), int(b)) for a, b in got}) == len(got)
    one = product_edges(rng.uniform(0, 10, (50, 2)), (100.0, 100.0), 1)
    assert len(one) == 50 * 49 // 2


@pytest.mark.parametrize("lam", [0.975, 0.5, 0.14])
@pytest.mark.parametrize("kind,cells", [("h", 8), ("f", 8), ("h", 3)])
def test_labeling_matches_oracle_energy_and_independent_cut(lam, kind, cells):
    # the engine cuts every grid cell on its own; the oracle runs BK once over
    # the whole graph (GCRANSAC.h:759-870): the labelings must be identical
    if kind == "h":
        corr, _, _, thr = S.problem_h(2500, 0.5, seed=11)
    else:
        corr, _, _, thr = S.problem_f(6000, 0.8, seed=12)
    sizes = (1280.0 / cells, 960.0 / cells, 1280.0 / cells, 960.0 / cells)
    edges = O.grid_edges(corr, sizes, cells)
    rng = np.random.default_rng(int(lam * 1000) + cells)
    sqt = (1.5 * thr) ** 2
    r2 = np.where(rng.random(corr.shape[0]) < 0.5, rng.uniform(0, 1.2 * sqt, corr.shape[0]),
                  rng.uniform(0, 30 * sqt, corr.shape[0]))
    r2[::17] = sqt                                        # exactly at the truncation
    got = product_labeling(r2, sqt, lam, corr, sizes, cells)
    unary, pair = labeling_energy(r2, sqt, lam, edges)
    ref = product_bk(unary, edges, pair)                  # whole-graph BK, product code
    assert np.array_equal(got, ref)
    assert np.array_equal(got, O.bk_energy(unary, edges, pair)[0])
    # pairwise terms change the labeling relative to the terminal test
    plain = (0.0 - (1.0 - lam) * (1.0 - np.clip(r2 / sqt, 0, 1))) < 0
    assert not np.array_equal(got, plain)
    # no better labeling one flip away (a local check of optimality)
    e_got = energy_of(got.astype(int), unary, edges, pair)
    for i in rng.choice(r2.size, 200, replace=False):
        x = got.astype(int)
        x[i] ^= 1
        assert energy_of(x, unary, edges, pair) >= e_got - 1e-9


def test_labeling_without_edges_is_the_terminal_test():
    rng = np.random.default_rng(2)
    sqt = 4.0
    r2 = rng.uniform(0, 8, 1000)
    r2[:5] = [0.0, sqt, np.nextafter(sqt, 0), np.nextafter(sqt, 9), 8.0]
    for lam in (0.0, 0.5, 0.975):
        got = product_labeling(r2, sqt, lam)
        q = np.clip(r2 / sqt, 0, 1)
        tr = np.where(r2 <= sqt, 0.0 - (1 - lam) * (1 - q), (1 - lam) * (1 - (1 - q)) - 0.0)
        assert np.array_equal(got, tr < 0)


def test_grid_cell_sizes_unknown_image_sizes():
    # an image size <= 0 (or not finite) falls back to that axis's extent of
    # the finite coordinates (max + 1, at least 1 px), divided by the cells
    from pygcransac import pygcransac as P

    rng = np.random.default_rng(5)
    corr = rng.uniform(0, 500, (300, 4))
    corr[7, 1] = np.nan
    corr[9, 2] = np.inf
    corr[:, 3] = -5.0                                        # no positive extent: 1 px
    got = P.grid_cell_sizes(corr, 0, 640, -1, float("nan"), 8)

    def ref(col, size):
        if size > 0 and np.isfinite(size):
            return size / 8
        v = corr[:, col][np.isfinite(corr[:, col])]
        return max(1.0, float(v.max()) + 1.0) / 8 if v.size else 1.0 / 8

    assert got == [ref(0, 640), ref(1, 0), ref(2, float("nan")), ref(3, -1)]
    assert P.grid_cell_sizes(np.zeros((0, 4)), 0, 0, 0, 0, 4) == [0.25] * 4


def test_two_point_cells_closed_form_equals_bk(tmp_path):
    # graphcut.h graphcut_pair (two-point cells, ~45 % of the cells at
    # configs[3]) decides BK's labeling without running it; checked against
    # graphcut_cell_bk on 2 M random cells with deliberate ties (residuals at
    # the truncated threshold, equal points, q in {0, 1/2, 1}, lambda 0 / 1)
    import os
    import subprocess

    here = os.path.dirname(os.path.abspath(__file__))
    exe = str(tmp_path / "gc_pair")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                           os.path.join(here, "cpp", "gc_pair.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout


def test_clique_cells_closed_form_equal_bk(tmp_path):
    # graphcut.h graphcut_clique (cells of >= 3 points with at most one source
    # node: nearly every cell at the default lambda) decides BK's labeling
    # without running it; checked against graphcut_cell_bk on 2 M random
    # cells of 3 .. 40 points with deliberate ties (residuals at the truncated
    # threshold, zero and equal residuals, NaN, lambda tiny / huge / 1)
    import os
    import subprocess

    here = os.path.dirname(os.path.abspath(__file__))
    exe = str(tmp_path / "gc_clique")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                           os.path.join(here, "cpp", "gc_clique.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout


def test_scheduled_labeling_equals_serial(tmp_path):
    # the engine's path: gc_schedule's cost-balanced jobs (largest cells
    # first, q written per cell) in schedule order, reversed, shuffled and on
    # 4 threads give the serial driver's labeling bit for bit (random
    # clustered 4-D grids, ties at the truncated threshold, 5 pool sizes)
    import os
    import subprocess

    here = os.path.dirname(os.path.abspath(__file__))
    exe = str(tmp_path / "gc_jobs")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-pthread",
                           os.path.join(here, "cpp", "gc_jobs.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout


def test_frozen_tie_fixtures():
    # tests/golden/graphcut_ties.json (tools/gen_gc_ties.py, written once, never
    # regenerated): labeling() calls whose energies tie on purpose (residuals
    # exactly at the truncated threshold, equal residuals, dyadic lambda); the
    # expected SINK sets come from the reference's reading rule (what_segment
    # with default SOURCE, GCRANSAC.h:865, graph.h:115-117) as the intersection
    # of all optimal labelings' sink sets over an exhaustive enumeration, with
    # no BK code involved.  Both BK implementations must return exactly them.
    import json
    import os

    with open(os.path.join(os.path.dirname(__file__), "golden", "graphcut_ties.json")) as f:
        cases = json.load(f)["cases"]
    assert sum(c["optimal_labelings"] >= 2 for c in cases) >= 15
    for c in cases:
        r2 = np.asarray(c["r2"], dtype=np.float64)
        pts = np.asarray(c["points"], dtype=np.float64)
        edges = np.asarray(c["edges"], dtype=np.uint32).reshape(-1, 2)
        assert np.array_equal(product_edges(pts, c["cell_size"], c["cells"]), edges), c["name"]
        expect = np.asarray(c["sink"], dtype=bool)
        got = product_labeling(r2, c["sqt"], c["lambda"], pts, c["cell_size"], c["cells"])
        assert np.array_equal(got, expect), c["name"]
        unary, pair = labeling_energy(r2, c["sqt"], c["lambda"], edges)
        assert np.array_equal(O.bk_energy(unary, edges, pair)[0], expect), c["name"]
        assert np.array_equal(product_bk(unary, edges, pair), expect), c["name"]
