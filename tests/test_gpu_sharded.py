"""One problem over several ranks (gcr_problem_run_sharded).

Two processes share the box's GPU (gloo carries the all-gather); each verifies
half of every chunk of slots and the replay runs on both.  The result must be
the single-rank result bit for bit, on both ranks, for the rectification,
homography and fundamental-matrix paths."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from gcr_testutil import bits
from pygcransac import _native as N
from pygcransac import distributed as D
from pygcransac import synthetic as S

pytestmark = pytest.mark.gpu


def _cases():
    fs, fo, _, _, ts, to = S.problem_m2(1500, 1200, seed=41)
    ch, _, _, th = S.problem_h(1000, 0.5, seed=42)
    cf, _, _, tf = S.problem_f(2000, 0.6, seed=43)
    common = dict(confidence=0.99, min_iteration_number=0, max_iteration_number=200000, seed=7)
    return [
        ("m2", N.SOLVER_SIFT22, fs, fo, dict(scale_residual_thresh=ts, orientation_residual_thresh=to, **common)),
        ("h", N.SOLVER_HOMOGRAPHY4, ch, None, dict(scale_residual_thresh=th, **common)),
        ("f", N.SOLVER_FUNDAMENTAL7, cf, None, dict(scale_residual_thresh=tf, **common)),
    ]


def _digest(res):
    H, masks, st, rec = res
    return dict(H=None if H is None else bits(H).tolist(), masks=[m.tolist() for m in masks],
                it=st["iteration_number"], lo=st["local_optimization_number"], gc=st["graph_cut_number"],
                hyp=st["hypotheses"], score=bits(st["score"]).tolist(), rec=bits(rec).tolist())


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        out = {}
        for name, solver, f0, f1, prm in _cases():
            out[name] = _digest(D.run_problem_sharded(solver, f0, f1, prm, rank=rank, world=world, dist=dist,
                                                      device=0))
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(out, fh)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(600)
def test_sharded_problem_equals_single_rank(tmp_path):
    if N.lib.gcr_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    outs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    for name, solver, f0, f1, prm in _cases():
        ref = json.loads(json.dumps(_digest(D.run_problem_sharded(solver, f0, f1, prm, device=0))))
        assert outs[0][name] == ref, name
        assert outs[1][name] == ref, name
        assert ref["H"] is not None and ref["hyp"] > 0


def test_single_rank_entry_equals_public_api():
    import pygcransac

    _, _, ch, _, prm = _cases()[1]
    H, masks, st, _ = D.run_problem_sharded(N.SOLVER_HOMOGRAPHY4, ch, None, prm, device=0)
    H2, m2, st2 = pygcransac.findHomography(ch, 0, 0, 0, 0, threshold=prm["scale_residual_thresh"], conf=0.99,
                                            spatial_coherence_weight=0.0, max_iters=200000, min_iters=0, seed=7,
                                            return_stats=True)
    assert np.array_equal(bits(H), bits(H2)) and np.array_equal(masks[0], m2)
    assert st["iteration_number"] == st2["iteration_number"]
