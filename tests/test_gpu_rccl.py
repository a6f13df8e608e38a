"""RCCL on the box: the "nccl" backend (RCCL on ROCm) with one rank per GPU.
The one-GPU box cannot host two RCCL ranks (one GPU per rank), so this runs a
world of 1 in a child process: process-group init over RCCL, the all-gather
callback of gcr_problem_run_sharded (distributed.make_allgather) on device
tensors, called the way the engine calls it, and bench.py's collectives
(all_reduce MAX / SUM, all_gather) on device tensors.  The two-rank exchange
itself is covered with gloo in test_gpu_sharded.py and test_distributed.py."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

from pygcransac import _native as N

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "graph-cut-ransac_amd")

CHILD = textwrap.dedent("""
    import ctypes as C, os, sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.environ["GCR_PKG"])
    from pygcransac import distributed as D
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + os.environ["GCR_PORT"], rank=0, world_size=1)
    try:
        assert dist.get_backend() == "nccl"
        dev = torch.device("cuda", 0)
        cb = D.make_allgather(dist, 1, dev)
        send = np.arange(5000, dtype=np.uint8) * 7
        recv = np.zeros_like(send)
        rc = cb(None, send.ctypes.data, recv.ctypes.data, send.size)
        assert rc == 0 and np.array_equal(send, recv), rc
        t = torch.tensor([1.5], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        m = torch.tensor([3.0], dtype=torch.float64, device=dev)
        dist.all_reduce(m, op=dist.ReduceOp.SUM)
        outs = [torch.empty(5, dtype=torch.float64, device=dev)]
        dist.all_gather(outs, torch.arange(5, dtype=torch.float64, device=dev))
        torch.cuda.synchronize()
        assert t.item() == 1.5 and m.item() == 3.0 and outs[0].tolist() == [0, 1, 2, 3, 4]
        dist.barrier()
        print("RCCL OK")
    finally:
        dist.destroy_process_group()
""")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_rccl_world1_allgather_callback_and_bench_collectives():
    if N.lib.gcr_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    env = dict(os.environ, GCR_PKG=PKG, GCR_PORT=str(_free_port()), MASTER_ADDR="127.0.0.1")
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0 and "RCCL OK" in out.stdout, out.stdout[-2000:] + out.stderr[-3000:]


# ---------------------------------------------------- engine communicator ----
# gcr_comm (RCCL inside libgcr): the hypothesis-sharded run's block summaries
# all-gathered by ncclAllGather on the device, behind the summary kernel (no
# Python callback, no host staging of the send side).  One GPU: a world of 1
# through that path, against the plain single-rank run, bit for bit -- with a
# one-member summary cap every chunk overflows, so the device continuation and
# the stop-slot locate go through the exchange too.
def _sharded_vs_single(kind, budget, monkeypatch, env):
    import numpy as np

    from gcr_testutil import bits
    from pygcransac import distributed as D
    from pygcransac import synthetic as S

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if kind == N.SOLVER_SIFT22:
        fs, fo, _, _, t0, t1 = S.problem_m2(1500, 1300, seed=61)
        f0, f1 = fs, fo
    elif kind == N.SOLVER_FUNDAMENTAL7:
        f0, _, _, t0 = S.problem_f(2500, 0.6, seed=63)
        f1, t1 = None, 0.0
    else:
        f0, _, t0 = S.problem_m1(2500, seed=64)
        f1, t1 = None, 0.0
    params = dict(scale_residual_thresh=t0, orientation_residual_thresh=t1, seed=11)
    if budget == "fixed":
        params.update(min_iteration_number=300_000, max_iteration_number=300_000)
    else:
        params.update(min_iteration_number=0, max_iteration_number=10**7, confidence=0.99)
    monkeypatch.setenv("GCR_EXCHANGE_LOG", "1")
    ref = D.run_problem_sharded(kind, f0, f1, params, 0, 1, device=0)
    ref_ev = N.exchange_log()
    comm = D.Comm(None, 0, 1, device=0)
    try:
        got = D.run_problem_sharded(kind, f0, f1, params, 0, 1, device=0, comm=comm)
        got_ev = N.exchange_log()
    finally:
        comm.close()
    monkeypatch.delenv("GCR_EXCHANGE_LOG")
    # the gcr_comm run issues its collectives (chunk issues and re-summaries)
    # in exactly the callback path's event sequence
    assert ref_ev and got_ev == ref_ev
    for k in env:
        monkeypatch.delenv(k)
    (Hr, mr, sr, rr), (Hg, mg, sg, rg) = ref, got
    assert all(np.array_equal(a, b) for a, b in zip(mr, mg))
    assert (Hr is None and Hg is None) or np.array_equal(bits(Hr), bits(Hg))
    for k in ("iteration_number", "hypotheses", "slots", "local_optimization_number", "graph_cut_number"):
        assert sr[k] == sg[k], k
    assert bits(sr["score"]) == bits(sg["score"])
    assert np.array_equal(bits(np.array(rr)), bits(np.array(rg)))


@pytest.mark.parametrize("kind", [N.SOLVER_SCALE3, N.SOLVER_SIFT22, N.SOLVER_FUNDAMENTAL7])
@pytest.mark.parametrize("budget", ["fixed", "adaptive"])
def test_engine_comm_world1_equals_single_rank(kind, budget, monkeypatch):
    if N.lib.gcr_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    _sharded_vs_single(kind, budget, monkeypatch, {})
    _sharded_vs_single(kind, budget, monkeypatch, {"GCR_SUMMARY_CAP": "1"})


# -------------------------------------------- engine communicator, world 2 ----
# Two ranks on two GPUs: fresh processes, each
# binding its own GPU before any HIP call, exchange over gcr_comm (RCCL inside
# libgcr) and over the gloo callback; both ranks must return the single-rank
# run bit for bit and log the same exchange sequence.  Runs only where two or
# more GPUs are visible (the driver's multi-GPU node); the one-GPU box skips.
CHILD2 = textwrap.dedent("""
    import json, os, sys
    import numpy as np
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ["GCR_EXCHANGE_LOG"] = "1"
    sys.path.insert(0, os.environ["GCR_PKG"])
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:" + os.environ["GCR_PORT"], rank=rank,
                            world_size=world)
    from pygcransac import _native as N
    from pygcransac import distributed as D
    from pygcransac import synthetic as S
    fs, fo, _, _, t0, t1 = S.problem_m2(1500, 1300, seed=61)
    params = dict(scale_residual_thresh=t0, orientation_residual_thresh=t1, seed=11,
                  min_iteration_number=0, max_iteration_number=10**7, confidence=0.99)
    out = {}
    comm = D.Comm(dist, rank, world, device=rank)
    try:
        H, masks, st, rec = D.run_problem_sharded(N.SOLVER_SIFT22, fs, fo, params, rank, world, device=rank,
                                                  comm=comm)
        out["comm_log"] = [list(map(int, x)) for x in N.exchange_log()]
    finally:
        comm.close()
    H2, masks2, st2, rec2 = D.run_problem_sharded(N.SOLVER_SIFT22, fs, fo, params, rank, world, dist=dist,
                                                  device=rank)
    out["cb_log"] = [list(map(int, x)) for x in N.exchange_log()]
    out["H"] = np.asarray(H).view(np.uint64).tolist()
    out["H2"] = np.asarray(H2).view(np.uint64).tolist()
    out["masks"] = [np.asarray(m).tolist() for m in masks]
    out["masks2"] = [np.asarray(m).tolist() for m in masks2]
    out["stats"] = {k: st[k] for k in ("iteration_number", "hypotheses", "slots", "local_optimization_number",
                                        "graph_cut_number")}
    out["score"] = float(st["score"]).hex()
    dist.barrier()
    dist.destroy_process_group()
    print("RESULT " + json.dumps(out))
""")


def _gpu_count_without_hip():
    # torch.cuda.device_count() does not initialise HIP on this image, so the
    # children below start on an untouched runtime either way
    import torch

    return torch.cuda.device_count()


@pytest.mark.timeout(600)
def test_engine_comm_world2_equals_single_rank():
    if _gpu_count_without_hip() < 2:
        pytest.skip("two GPUs needed for a world-2 RCCL run (this box has one)")
    import json

    import numpy as np

    port = str(_free_port())
    procs = []
    for r in range(2):
        env = dict(os.environ, GCR_PKG=PKG, GCR_PORT=port, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1")
        procs.append(subprocess.Popen([sys.executable, "-c", CHILD2], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    res = []
    for p in procs:
        o, e = p.communicate(timeout=540)
        assert p.returncode == 0, o[-2000:] + e[-3000:]
        res.append(json.loads(o.split("RESULT ", 1)[1]))
    # the single-rank run in this process
    from pygcransac import distributed as D
    from pygcransac import synthetic as S

    fs, fo, _, _, t0, t1 = S.problem_m2(1500, 1300, seed=61)
    params = dict(scale_residual_thresh=t0, orientation_residual_thresh=t1, seed=11,
                  min_iteration_number=0, max_iteration_number=10**7, confidence=0.99)
    H, masks, st, _ = D.run_problem_sharded(N.SOLVER_SIFT22, fs, fo, params, 0, 1, device=0)
    for r in res:
        assert r["comm_log"] and r["comm_log"] == r["cb_log"] == res[0]["comm_log"]
        assert r["H"] == r["H2"] == np.asarray(H).view(np.uint64).tolist()
        assert r["masks"] == r["masks2"] == [np.asarray(m).tolist() for m in masks]
        assert r["stats"] == {k: st[k] for k in r["stats"]}
        assert r["score"] == float(st["score"]).hex()
