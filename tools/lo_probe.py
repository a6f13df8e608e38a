#!/usr/bin/env python3
"""Wall time of one small-batch scoring launch (k_lo_chain through
gcr_debug_score, GCR_DEBUG_SCORER=small, synchronised) for 1 and 50 models of
the M2 workload (5000 + 5000 features), median of 40 calls.  Run once per
setting (GCR_PROBE bits 8: no fold, 9: no residual evaluation -- timing
probes, results invalid; GCR_LO_FOLD=seq: the one-lane fold)."""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "graph-cut-ransac_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ["GCR_DEBUG_SCORER"] = "small"

from gcr_testutil import Problem  # noqa: E402
from pygcransac import _native as N  # noqa: E402
from pygcransac import synthetic as S  # noqa: E402

fs, fo, _, _, t0, t1 = S.problem_m2(5000, 5000, seed=20251121)
prob = Problem(N.SOLVER_SIFT22, fs, fo)
inc, models = prob.generate(7, 0, 4096)
live = models[inc <= 101]
# LO-like models: the hypotheses with the most inliers (LO trials and refits
# score good models: ~5000 inliers to fold, not a random hypothesis's few)
n0, n1, _, _, _ = prob.score_raw(live, t0, t1)
order = sorted(range(len(live)), key=lambda i: -(int(n0[i]) + int(n1[i])))
live = live[order[:64]]
print("inliers of the chosen models:", int(n0[order[0]]) + int(n1[order[0]]), "..",
      int(n0[order[49]]) + int(n1[order[49]]), flush=True)
tag = os.environ.get("TAG", "")
for nm in (1, 50):
    ms = live[:nm]
    for _ in range(5):
        prob.score_raw(ms, t0, t1)
    ts = []
    for _ in range(40):
        a = time.perf_counter()
        prob.score_raw(ms, t0, t1)
        ts.append((time.perf_counter() - a) * 1e6)
    print(f"{tag:10s} models {nm:3d}: median {statistics.median(ts):7.1f} us  min {min(ts):7.1f} us", flush=True)
