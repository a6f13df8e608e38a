"""Problem sharding and the final-model gather (pygcransac/distributed.py) on
CPU: LPT assignment properties and a world_size-2 gloo run of solve_sharded
with a deterministic stand-in solver (the GPU engine is exercised per rank
by the gpu tests and bench.py)."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from pygcransac import distributed as D


def _problems(n, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = int(rng.integers(3, 40))
        out.append(dict(kind="scale_only", features=rng.normal(size=(k, 3)), scale_residual_thresh=0.05,
                        max_iteration_number=int(rng.integers(100, 5000)), tag=i))
    return out


def _fake_solve(pr):
    f = np.asarray(pr["features"])
    if pr["tag"] % 7 == 3:         # some problems fail (no model), as the estimator can
        return dict(H=None, model=None, num_inliers=0, stats=dict(iteration_number=5, hypotheses=0))

    class M:
        x0, y0, s = 0.0, 0.0, 1.0
        h7, h8, alpha, phi = float(f[:, 0].sum()), float(f[:, 1].sum()), float(pr["tag"]), 0.25

    H = np.eye(3)
    H[2, :2] = [M.h7, M.h8]
    return dict(H=H, model=M, num_inliers=f.shape[0], stats=dict(iteration_number=pr["tag"] + 1, hypotheses=7))


def test_lpt_covers_every_problem_once_and_balances():
    costs = [D.problem_cost(p) for p in _problems(101, seed=3)]
    for world in (1, 2, 3, 8):
        shares = D.assign_lpt(costs, world)
        flat = sorted(i for s in shares for i in s)
        assert flat == list(range(len(costs)))
        loads = [sum(costs[i] for i in s) for s in shares]
        # LPT bound: makespan <= 4/3 OPT; OPT >= max(mean load, largest job)
        assert max(loads) <= 4.0 / 3.0 * max(sum(costs) / world, max(costs)) + 1e-9
        assert D.assign_lpt(costs, world) == shares          # deterministic


def test_record_roundtrip_and_failures():
    for p in _problems(10):
        r = _fake_solve(p)
        rec = D.decode_record(D.encode_result(r))
        if r["model"] is None:
            assert rec["H"] is None and rec["num_inliers"] == 0
        else:
            assert np.array_equal(rec["H"], r["H"]) and rec["model"]["alpha"] == r["model"].alpha
    assert D.decode_record(D.encode_result(None)) is None


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        recs, local = D.solve_sharded(_problems(23, seed=1), _fake_solve, rank=rank, world=world, dist=dist)
        payload = dict(local=sorted(local), recs=[None if r is None else
                                                  dict(n=r["num_inliers"], h7=r["model"]["h7"], it=r["iteration_number"])
                                                  for r in recs])
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
            json.dump(payload, f)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(120)
def test_solve_sharded_gloo_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    outs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    # every rank holds every problem's record, identical across ranks
    assert outs[0]["recs"] == outs[1]["recs"]
    # ranks solved disjoint shares covering all problems (no duplicated work)
    assert sorted(outs[0]["local"] + outs[1]["local"]) == list(range(23))
    assert not set(outs[0]["local"]) & set(outs[1]["local"])
    # records equal a single-process solve
    ref, _ = D.solve_sharded(_problems(23, seed=1), _fake_solve)
    exp = [None if r is None else dict(n=r["num_inliers"], h7=r["model"]["h7"], it=r["iteration_number"])
           for r in ref]
    assert outs[0]["recs"] == exp


# --------------------------------------- one problem, many ranks (e row 2) ---
def _allgather_worker(rank, world, port, outdir):
    import ctypes as C

    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        cb = D.make_allgather(dist, world)
        nbytes = 1000 + 24 * 7
        send = (np.arange(nbytes) * (rank + 3) % 251).astype(np.uint8)
        recv = np.zeros(world * nbytes, dtype=np.uint8)
        rcs = [cb(None, send.ctypes.data, recv.ctypes.data, nbytes) for _ in range(3)]   # repeated exchanges
        with open(os.path.join(outdir, f"ag{rank}.json"), "w") as f:
            json.dump(dict(rcs=rcs, recv=recv.tolist()), f)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_allgather_callback_gloo_world2(tmp_path):
    # the exchange gcr_problem_run_sharded calls through its C function pointer
    world = 2
    mp.spawn(_allgather_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    nbytes = 1000 + 24 * 7
    exp = np.concatenate([(np.arange(nbytes) * (r + 3) % 251).astype(np.uint8) for r in range(world)]).tolist()
    for r in range(world):
        out = json.load(open(tmp_path / f"ag{r}.json"))
        assert out["rcs"] == [0, 0, 0]
        assert out["recv"] == exp


def test_problem_defaults_are_the_direct_entry_points_defaults():
    # gpu_solver and batch_solver fill omitted keys from one per-kind table,
    # which must equal the defaults of the direct call each kind maps to
    import inspect

    import pygcransac as P
    from pygcransac import distributed as D

    sig = inspect.signature(P.findHomography).parameters
    corr = D.problem_settings({"kind": "homography"})
    assert corr == D.problem_settings({"kind": "fundamental"})
    assert corr["confidence"] == sig["conf"].default
    assert corr["spatial_coherence_weight"] == sig["spatial_coherence_weight"].default
    assert corr["max_iteration_number"] == sig["max_iters"].default
    assert corr["min_iteration_number"] == sig["min_iters"].default
    assert corr["max_local_optimization_number"] == sig["lo_number"].default
    sig = inspect.signature(P.findRectifyingHomographySIFT).parameters
    for kind in ("sift", "scale_only", "scale_only_original"):
        rect = D.problem_settings({"kind": kind})
        for k in ("spatial_coherence_weight", "min_iteration_number", "max_iteration_number",
                  "max_local_optimization_number"):
            assert rect[k] == sig[k].default, (kind, k)
        assert rect["confidence"] == 0.95          # settings.h:60, fixed by the reference
    assert D.problem_settings({"kind": "sift", "seed": 5, "confidence": 0.99})["seed"] == 5
