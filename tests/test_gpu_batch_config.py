"""BASELINE configs[4] under test (run on an MI355X: pytest -m gpu): the
1024-problem mixed batch bench.py's `--workload batch` measures (homography /
fundamental / hybrid / scale-only, N ~ U{1000..10000}, 50 % outliers,
confidence 0.99), solved in ONE gcr_solve_batch call on one GPU with the
bench's 8 host threads, against one-by-one gpu_solver calls on a seeded subset
of 64 problems (bitwise digests: H, masks, inlier counts, run statistics).
No reference counterpart (the reference binds single problems only,
bindings.cpp:315-399); the per-problem results are pinned to the oracle by the
end-to-end parity suites."""
import os
import sys

import numpy as np
import pytest

from pygcransac import _native as N
from pygcransac import distributed as D

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    if N.lib.gcr_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    N.context(0)


def _digest(res):
    H = res["H"]
    return (None if H is None else np.asarray(H, dtype=np.float64).tobytes(),
            tuple(np.asarray(m, dtype=bool).tobytes() for m in res["masks"]),
            int(res["num_inliers"]),
            int(res["stats"]["iteration_number"]), int(res["stats"]["hypotheses"]),
            int(res["stats"]["local_optimization_number"]), int(res["stats"]["graph_cut_number"]))


def test_configs4_batch_of_1024_matches_one_by_one_calls():
    problems = bench.batch_problems(1024)
    out = D.batch_solver(0, 8)(problems)
    assert len(out) == len(problems)
    kinds = {}
    for pr, r in zip(problems, out):
        kinds[pr["kind"]] = kinds.get(pr["kind"], 0) + 1
        assert r["num_inliers"] > 0, pr["kind"]                 # 50 % outliers: every problem is solved
        assert np.all(np.isfinite(r["H"]))
        n = sum(np.asarray(f).shape[0] for k, f in pr.items()
                if k in ("features", "scale_features", "orientation_features", "correspondences"))
        assert sum(m.size for m in r["masks"]) == n
        assert sum(int(m.sum()) for m in r["masks"]) == r["num_inliers"]
    assert kinds == {"homography": 256, "fundamental": 256, "sift": 256, "scale_only": 256}
    subset = np.random.default_rng(2024).choice(len(problems), 64, replace=False)
    solve = D.gpu_solver(0)
    for i in sorted(subset):
        assert _digest(solve(problems[i])) == _digest(out[i]), (i, problems[i]["kind"])


def test_batch_and_direct_solvers_share_defaults_per_kind():
    # a problem dict without the optional keys gives the same result through
    # both solve paths (the defaults come from one per-kind table)
    from pygcransac import synthetic as S

    c, _, _, thr = S.problem_h(1500, 0.5, seed=71)
    f, _, thr_s = S.problem_m1(1200, seed=72)
    probs = [dict(kind="homography", correspondences=c, threshold=thr),
             dict(kind="scale_only", features=f, scale_residual_thresh=thr_s)]
    many = D.batch_solver(0, 2)(probs)
    solve = D.gpu_solver(0)
    for pr, r in zip(probs, many):
        assert _digest(solve(pr)) == _digest(r), pr["kind"]
