"""Graph-cut LO with pairwise terms, end to end on the GPU (pytest -m gpu):
findHomography / findFundamentalMatrix with spatial_coherence_weight > 0 and a
neighbourhood grid over (x1, y1, x2, y2) against the oracle run with the same
grid (GCRANSAC.h:759-870 labeling, grid_neighborhood_graph.h:229-301), bitwise:
masks, the returned matrix and the run statistics.  Parity with any
reference is unpinned for these estimators (absent from the fork, finding
0.1); the labeling pieces themselves are pinned in tests/test_graphcut.py."""
import numpy as np
import pytest

import oracle_ffi as O
import pygcransac
from gcr_testutil import bits
from pygcransac import _native as N
from pygcransac import pygcransac as P
from pygcransac import synthetic as S

pytestmark = pytest.mark.gpu

H1, W1, H2, W2 = 960, 1280, 960, 1280


@pytest.fixture(scope="module", autouse=True)
def _device():
    if N.lib.gcr_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    N.context(0)


def _run(kind, corr, thr, lam, cells, seed, min_it=50, max_it=3000):
    fn = pygcransac.findHomography if kind == "h" else pygcransac.findFundamentalMatrix
    M, mask, st = fn(corr, H1, W1, H2, W2, threshold=thr, conf=0.99, spatial_coherence_weight=lam,
                     max_iters=max_it, min_iters=min_it, neighborhood_size=cells, seed=seed, device=0,
                     return_stats=True)
    sizes = P.grid_cell_sizes(corr, H1, W1, H2, W2, cells) if cells else (0, 0, 0, 0)
    ofn = O.find_homography if kind == "h" else O.find_fundamental
    ref = ofn(corr, thr, lam=lam, min_it=min_it, max_it=max_it, confidence=0.99, seed=seed, cell_size=sizes,
              cell_number=cells)
    return M, mask, st, ref


@pytest.mark.parametrize("kind,n,outl,seed", [("h", 2000, 0.5, 3), ("h", 5000, 0.5, 4), ("f", 3000, 0.5, 5),
                                              ("f", 4000, 0.7, 6)])
@pytest.mark.parametrize("lam", [0.975, 0.5])
def test_graph_cut_lo_with_pairwise_terms_matches_oracle(kind, n, outl, seed, lam):
    if kind == "h":
        corr, _, _, thr = S.problem_h(n, outl, seed=100 + seed)
    else:
        corr, _, _, thr = S.problem_f(n, outl, seed=100 + seed)
    M, mask, st, ref = _run(kind, corr, thr, lam, 8, seed)
    assert np.array_equal(mask, ref["mask"])
    assert np.array_equal(bits(M), bits(ref["H"]))
    for k in ("iteration_number", "local_optimization_number", "graph_cut_number"):
        assert st[k] == ref["stats"][k], k
    assert st["graph_cut_number"] > 0


def test_grid_sizes_from_data_and_empty_grid():
    corr, _, _, thr = S.problem_h(1500, 0.5, seed=77)
    # image sizes unknown (0): the grid spans the data's extent
    M, mask, st = pygcransac.findHomography(corr, 0, 0, 0, 0, threshold=thr, spatial_coherence_weight=0.975,
                                            max_iters=2000, min_iters=50, seed=2, device=0, return_stats=True)
    sizes = P.grid_cell_sizes(corr, 0, 0, 0, 0, 8)
    ref = O.find_homography(corr, thr, lam=0.975, min_it=50, max_it=2000, confidence=0.99, seed=2,
                            cell_size=sizes, cell_number=8)
    assert np.array_equal(mask, ref["mask"]) and np.array_equal(bits(M), bits(ref["H"]))
    # neighborhood_size=0: the empty grid, identical to lambda = 0 labeling
    a = pygcransac.findHomography(corr, H1, W1, H2, W2, threshold=thr, spatial_coherence_weight=0.975,
                                  max_iters=2000, min_iters=50, neighborhood_size=0, seed=2, device=0)
    b = pygcransac.findHomography(corr, H1, W1, H2, W2, threshold=thr, spatial_coherence_weight=0.0,
                                  max_iters=2000, min_iters=50, neighborhood_size=0, seed=2, device=0)
    assert np.array_equal(a[1], b[1]) and np.array_equal(bits(a[0]), bits(b[0]))


def test_rectification_rejects_a_grid():
    import ctypes as C

    f, _, thr = S.problem_m1(300, seed=1)
    p = N.default_params()
    p.scale_residual_thresh = thr
    p.cell_number = 8
    p.cell_size[:] = [10.0, 10.0, 10.0, 10.0]
    m = np.zeros(300, np.uint8)
    H = np.zeros(9)
    rc = N.lib.gcr_rect_scale_only(N.context(0), np.ascontiguousarray(f).ctypes.data_as(C.POINTER(C.c_double)),
                                   300, C.byref(p), 0, m.ctypes.data_as(C.POINTER(C.c_uint8)),
                                   H.ctypes.data_as(C.POINTER(C.c_double)), None, None)
    assert rc == N.GCR_EINVAL


def _direct_h(corr, thr, cell_size, cells=8, seed=2):
    """gcr_find_homography with explicit gcr_params grid fields."""
    import ctypes as C

    c = np.ascontiguousarray(corr, dtype=np.float64)
    p = N.default_params()
    p.scale_residual_thresh = thr
    p.spatial_coherence_weight = 0.975
    p.min_iteration_number, p.max_iteration_number = 50, 2000
    p.confidence, p.seed = 0.99, seed
    p.cell_number = cells
    p.cell_size[:] = list(cell_size)
    mask = np.zeros(c.shape[0], np.uint8)
    M = np.zeros(9)
    rc = N.lib.gcr_find_homography(N.context(0), c.ctypes.data, c.shape[0], C.byref(p), mask.ctypes.data,
                                   M.ctypes.data, None)
    return rc, mask.view(bool), M.reshape(3, 3)


def test_zero_cell_sizes_are_taken_from_the_data():
    # ABI 5: cell_size[d] == 0 -> the column's largest finite coordinate + 1
    # over the cells, computed by the engine; equal to the Python sizing
    # (grid_cell_sizes) the direct entry point applies, so the run is the
    # oracle's with those sizes bit for bit.  One known axis mixed in.
    corr, _, _, thr = S.problem_h(1800, 0.5, seed=91)
    sizes = P.grid_cell_sizes(corr, 0, W1, 0, 0, 8)
    rc, mask, M = _direct_h(corr, thr, [W1 / 8.0, 0.0, 0.0, 0.0])
    # grid_cell_sizes' argument order is (h1, w1, h2, w2); its sizes (w1, h1, w2, h2)
    assert rc > 0 and sizes[0] == W1 / 8.0
    ref = O.find_homography(corr, thr, lam=0.975, min_it=50, max_it=2000, confidence=0.99, seed=2,
                            cell_size=sizes, cell_number=8)
    assert np.array_equal(mask, ref["mask"]) and np.array_equal(bits(M), bits(ref["H"]))
    rc2, mask2, M2 = _direct_h(corr, thr, sizes)
    assert rc2 == rc and np.array_equal(mask2, mask) and np.array_equal(bits(M2), bits(M))


def test_negative_or_nonfinite_cell_sizes_are_rejected():
    corr, _, _, thr = S.problem_h(300, 0.5, seed=92)
    for bad in ([-1.0, 10.0, 10.0, 10.0], [10.0, float("inf"), 10.0, 10.0], [10.0, 10.0, float("nan"), 10.0]):
        rc, _, _ = _direct_h(corr, thr, bad)
        assert rc == N.GCR_EINVAL, bad
