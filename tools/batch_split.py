"""Where the configs[4] batch's wall time goes: the Python item fill, the
gcr_solve_batch call itself and the read-back (bench.py --workload batch's
timed region, split).  Usage: python tools/batch_split.py [problems] [threads]"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "graph-cut-ransac_amd"))

import bench  # noqa: E402
from pygcransac import _native as N, distributed as D  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
probs = bench.batch_problems(n)
real = N.lib
t_call = []


class Timed:
    def __getattr__(self, k):
        f = getattr(real, k)
        if k != "gcr_solve_batch":
            return f

        def g(*a):
            t = time.perf_counter()
            rc = f(*a)
            t_call.append(time.perf_counter() - t)
            return rc
        return g


N.lib = Timed()
sm = D.batch_solver(0, threads)
sm(probs[:16])
for rep in range(3):
    t_call.clear()
    t = time.perf_counter()
    D.solve_sharded(probs, rank=0, world=1, solve_many=sm)
    tot = time.perf_counter() - t
    print(f"job {tot * 1e3:.1f} ms  gcr_solve_batch {t_call[0] * 1e3:.1f} ms  python {1e3 * (tot - t_call[0]):.1f} ms  "
          f"{n / tot:.0f} problems/s", flush=True)
