"""Independent problems across the GPUs of a node.

One process per GPU (torchrun); problems are independent GCRANSAC runs, so the
data path needs no collective at all: each rank solves its share on its own
device, and the final models (a fixed-size record per problem, a few hundred
bytes) are gathered with ONE all_gather -- RCCL over xGMI on the "nccl"
backend, gloo on CPU.  Inlier masks stay with the rank that computed them.

Extension module: the reference has no batch entry point
(bindings.cpp:315-399 binds single problems only).
"""
from __future__ import annotations

import heapq
from typing import Callable, Optional, Sequence

import numpy as np

# record layout: [valid, num_inliers, H (9), model x0 y0 s h7 h8 alpha phi (7),
#                 iteration_number, hypotheses]
RECORD = 20


# Defaults of a problem dict's optional keys, per kind: exactly the defaults of
# the direct entry point the kind maps to (bindings.cpp:366-396 for the
# rectification functions -- the reference fixes confidence at 0.95,
# settings.h:60; pygcransac.findHomography / findFundamentalMatrix for the
# correspondence kinds), so gpu_solver and batch_solver agree with each other
# and with the direct calls when a key is omitted.
_RECT_DEFAULTS = dict(spatial_coherence_weight=0.0, min_iteration_number=10000, max_iteration_number=10000,
                      max_local_optimization_number=50, confidence=0.95, seed=0)
_CORR_DEFAULTS = dict(spatial_coherence_weight=0.975, min_iteration_number=50, max_iteration_number=10000,
                      max_local_optimization_number=50, confidence=0.99, seed=0, image_sizes=(0, 0, 0, 0),
                      neighborhood_size=8)


def problem_settings(problem: dict) -> dict:
    """The run settings of a problem dict: its own keys over the defaults of
    its kind (see _RECT_DEFAULTS / _CORR_DEFAULTS)."""
    base = _CORR_DEFAULTS if problem["kind"] in ("homography", "fundamental") else _RECT_DEFAULTS
    return {k: problem.get(k, v) for k, v in base.items()}


def problem_cost(problem: dict) -> float:
    """Estimated cost of a problem: feature count x hypotheses budget."""
    n = sum(np.asarray(problem[k]).shape[0]
            for k in ("features", "scale_features", "orientation_features", "correspondences")
            if k in problem and problem[k] is not None)
    return float(n) * float(problem_settings(problem)["max_iteration_number"])


def assign_lpt(costs: Sequence[float], world: int) -> list[list[int]]:
    """Longest-processing-time-first assignment of problems to `world` ranks.

    Deterministic (ties by problem index, then rank), every problem appears
    exactly once, and each rank's list is in increasing problem order."""
    if world < 1:
        raise ValueError("world must be >= 1")
    heap = [(0.0, r) for r in range(world)]
    shares: list[list[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda i: (-float(costs[i]), i)):
        load, r = heapq.heappop(heap)
        shares[r].append(i)
        heapq.heappush(heap, (load + float(costs[i]), r))
    return [sorted(s) for s in shares]


def encode_result(result) -> np.ndarray:
    """Fixed-size float64 record of one estimator result (see RECORD)."""
    rec = np.zeros(RECORD)
    if result is None:
        return rec
    H, model, num_inliers, stats = result.get("H"), result.get("model"), result.get("num_inliers", 0), \
        result.get("stats") or {}
    rec[0] = 1.0
    rec[1] = float(num_inliers)
    if H is not None:
        rec[2:11] = np.asarray(H, dtype=np.float64).ravel()
    if model is not None:
        rec[11:18] = [float(getattr(model, k, 0.0)) for k in ("x0", "y0", "s", "h7", "h8", "alpha", "phi")]
    rec[18] = float(stats.get("iteration_number", 0))
    rec[19] = float(stats.get("hypotheses", 0))
    return rec


def decode_record(rec: np.ndarray) -> Optional[dict]:
    if rec[0] == 0.0:
        return None
    return dict(num_inliers=int(rec[1]), H=None if not np.any(rec[2:11]) else rec[2:11].reshape(3, 3).copy(),
                model=dict(zip(("x0", "y0", "s", "h7", "h8", "alpha", "phi"), rec[11:18].tolist())),
                iteration_number=int(rec[18]), hypotheses=int(rec[19]))


def solve_sharded(problems: Sequence[dict], solve: Optional[Callable[[dict], dict]] = None, rank: int = 0,
                  world: int = 1, dist=None, device=None,
                  solve_many: Optional[Callable[[list], list]] = None) -> tuple[list[Optional[dict]], dict]:
    """Solve this rank's LPT share with `solve(problem) -> result dict`
    (keys H, model, num_inliers, stats, plus anything rank-local such as masks)
    or, for the whole share at once, `solve_many(problems) -> [result dict]`
    (e.g. `batch_solver`), then gather every problem's record to every rank
    with one all_gather.

    Returns (records in problem order -- all ranks, local results by index)."""
    shares = assign_lpt([problem_cost(p) for p in problems], world)
    mine = shares[rank]
    if solve_many is not None:
        local = dict(zip(mine, solve_many([problems[i] for i in mine])))
    else:
        local = {i: solve(problems[i]) for i in mine}
    cap = max(1, max(len(s) for s in shares))
    buf = np.zeros((cap, RECORD))
    for j, i in enumerate(mine):
        buf[j] = encode_result(local[i])
    if world == 1 or dist is None:
        gathered = [buf]
    else:
        import torch

        t = torch.from_numpy(buf)
        if device is not None:
            t = t.to(device)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)                  # the only collective
        gathered = [o.cpu().numpy() for o in outs]
    records: list[Optional[dict]] = [None] * len(problems)
    for r, share in enumerate(shares):
        for j, i in enumerate(share):
            records[i] = decode_record(gathered[r][j])
    return records, local


def gpu_solver(device: int) -> Callable[[dict], dict]:
    """solve() for solve_sharded that runs the MI355X engine on `device`.

    A problem is a dict with kind "sift" (scale_features, orientation_features,
    scale_residual_thresh, orientation_residual_thresh), "scale_only" /
    "scale_only_original" (features, scale_residual_thresh) or "homography" /
    "fundamental" (correspondences (N, 4), threshold), plus optional
    spatial_coherence_weight, min/max_iteration_number,
    max_local_optimization_number, seed, confidence."""
    from . import pygcransac as P

    def solve(pr: dict) -> dict:
        st = problem_settings(pr)
        if pr["kind"] in ("homography", "fundamental"):
            fn = P.findHomography if pr["kind"] == "homography" else P.findFundamentalMatrix
            out = fn(pr["correspondences"], *st["image_sizes"], threshold=pr["threshold"],
                     conf=st["confidence"], spatial_coherence_weight=st["spatial_coherence_weight"],
                     max_iters=st["max_iteration_number"], min_iters=st["min_iteration_number"],
                     lo_number=st["max_local_optimization_number"], neighborhood_size=st["neighborhood_size"],
                     seed=st["seed"], device=device, return_stats=True)
            M, mask, stats = out
            return dict(H=M, model=None, num_inliers=int(mask.sum()), stats=stats, masks=(mask,))
        common = [st["spatial_coherence_weight"], st["min_iteration_number"], st["max_iteration_number"],
                  st["max_local_optimization_number"]]
        kw = dict(seed=st["seed"], confidence=st["confidence"], device=device, return_stats=True)
        if pr["kind"] == "sift":
            out = P.findRectifyingHomographySIFT(pr["scale_features"], pr["orientation_features"],
                                                 pr["scale_residual_thresh"], pr["orientation_residual_thresh"],
                                                 *common, **kw)
            H, sm, om, model, stats = out
            return dict(H=H, model=model, num_inliers=int(sm.sum() + om.sum()), stats=stats, masks=(sm, om))
        fn = P.findRectifyingHomographyScaleOnlyOriginal if pr["kind"] == "scale_only_original" \
            else P.findRectifyingHomographyScaleOnly
        out = fn(pr["features"], pr["scale_residual_thresh"], *common, **kw)
        if len(out) == 3:          # (None, inliers, stats) on failure
            return dict(H=None, model=None, num_inliers=0, stats=out[-1], masks=(out[1],))
        H, m, model, stats = out
        return dict(H=H, model=model, num_inliers=int(m.sum()), stats=stats, masks=(m,))

    return solve


# ------------------------------------------------ one problem, many ranks ----
def make_allgather(dist, world: int, device=None):
    """ctypes all-gather callback for gcr_problem_run_sharded over a
    torch.distributed group: RCCL (device tensors) on "nccl", gloo on CPU.
    Keep the returned object alive for the duration of the call."""
    import ctypes as C

    import torch

    from . import _native as N

    def fn(_user, send, recv, nbytes):
        try:
            src = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(send))
            t = torch.from_numpy(src.copy())
            if device is not None:
                t = t.to(device)
            outs = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(outs, t)
            o = torch.cat(outs).cpu().numpy()
            C.memmove(recv, o.ctypes.data, world * nbytes)
            return 0
        except Exception:          # noqa: BLE001 -- reported to the engine as a failed exchange
            return -1

    return N.ALLGATHER_FN(fn)


class Comm:
    """An engine communicator rank (gcr_comm: RCCL over xGMI, one process per
    GPU) for gcr_problem_run_comm: the block summaries are all-gathered on the
    device by ncclAllGather, behind the summary kernel, with no Python in the
    exchange.  Rank 0 draws the RCCL unique id; `dist` (torch.distributed,
    any backend) broadcasts it once.  Collective: every rank constructs it."""

    def __init__(self, dist, rank: int, world: int, device: Optional[int] = None):
        import ctypes as C

        from . import _native as N

        self._N = N
        ident = (C.c_uint8 * 128)()
        if rank == 0:
            N.check(N.lib.gcr_comm_unique_id(ident))
        obj = [bytes(ident)]
        if dist is not None and world > 1:
            dist.broadcast_object_list(obj, src=0)
        buf = (C.c_uint8 * 128).from_buffer_copy(obj[0])
        h = C.c_void_p()
        N.check(N.lib.gcr_comm_create(N.context(device), rank, world, buf, C.byref(h)))
        self.h = h.value
        self.rank, self.world = rank, world

    def close(self):
        if getattr(self, "h", None):
            self._N.lib.gcr_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def run_problem_sharded(solver: int, f0, f1=None, params: Optional[dict] = None, rank: int = 0, world: int = 1,
                        dist=None, device: Optional[int] = None, coll_device=None, comm: Optional[Comm] = None):
    """One estimator problem over `world` ranks.

    Every rank calls this with the same inputs; each verifies its block of
    every chunk of slots on its own GPU and the chunks are all-gathered, so
    every rank returns the single-rank result bit for bit.  `params` holds
    gcr_params fields (scale_residual_thresh, confidence, seed, ...).  With
    `comm` (a Comm) the exchange runs inside the engine (ncclAllGather on the
    device); otherwise through `dist` in a Python callback (gloo or RCCL).
    Returns (H (3, 3) or None, masks tuple, stats dict, rect model record)."""
    import ctypes as C

    from . import _native as N

    f0 = np.ascontiguousarray(f0, dtype=np.float64)
    f1 = None if f1 is None else np.ascontiguousarray(f1, dtype=np.float64)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    ctx = N.context(device)
    h = C.c_void_p()
    N.check(N.lib.gcr_problem_create(ctx, solver, dp(f0), f0.shape[0], dp(f1) if f1 is not None else None,
                                     0 if f1 is None else f1.shape[0], C.byref(h)))
    try:
        p = N.default_params()
        for k, v in (params or {}).items():
            setattr(p, k, v)
        m0 = np.zeros(f0.shape[0], dtype=np.uint8)
        m1 = np.zeros(0 if f1 is None else f1.shape[0], dtype=np.uint8)
        H = np.zeros(9)
        model = N.RectModel()
        st = N.Stats()
        u8 = C.POINTER(C.c_uint8)
        if comm is not None:
            rc = N.lib.gcr_problem_run_comm(h, C.byref(p), comm.h, m0.ctypes.data_as(u8),
                                            m1.ctypes.data_as(u8) if f1 is not None else None, dp(H),
                                            C.byref(model), C.byref(st))
        else:
            cb = make_allgather(dist, world, coll_device) if world > 1 else N.ALLGATHER_FN(0)
            rc = N.lib.gcr_problem_run_sharded(h, C.byref(p), rank, world, cb, None, m0.ctypes.data_as(u8),
                                               m1.ctypes.data_as(u8) if f1 is not None else None, dp(H),
                                               C.byref(model), C.byref(st))
        n = N.check(rc)
    finally:
        N.lib.gcr_problem_destroy(h)
    masks = (m0.astype(bool),) if f1 is None else (m0.astype(bool), m1.astype(bool))
    rec = [model.x0, model.y0, model.s, model.h7, model.h8, model.alpha, model.phi]
    return (H.reshape(3, 3) if n > 0 else None), masks, st.as_dict(), rec


# ------------------------------------------------ native batch (one device) --
_SOLVERS = {"scale_only": 0, "scale_only_original": 1, "sift": 2, "homography": 3, "fundamental": 4}


def batch_solver(device: int = 0, concurrency: int = 4) -> Callable[[list], list]:
    """solve_many() for solve_sharded: the rank's share in ONE gcr_solve_batch
    call (`concurrency` host threads, a HIP stream and workspace each, so host
    phases of one problem overlap kernels of another).  Problem dicts as for
    gpu_solver."""
    import ctypes as C

    from . import _native as N
    from . import pygcransac as P

    # The items are filled and read column-wise through a numpy view of the
    # ctypes array (pointer fields as 64-bit addresses): per-item ctypes
    # attribute traffic cost ~60 ms of Python per 1024 problems, a fifth of
    # the configs[4] job.
    B = N.BatchItem
    fields = dict(solver=(np.int32, B.solver.offset), f0=(np.uint64, B.f0.offset), n0=(np.uint64, B.n0.offset),
                  f1=(np.uint64, B.f1.offset), n1=(np.uint64, B.n1.offset),
                  params=(np.dtype(N.Params), B.params.offset), mask0_out=(np.uint64, B.mask0_out.offset),
                  mask1_out=(np.uint64, B.mask1_out.offset), H_out=((np.float64, 9), B.H_out.offset),
                  stats_out=(np.dtype(N.Stats), B.stats_out.offset), result=(np.int32, B.result.offset))
    item_dt = np.dtype(dict(names=list(fields), formats=[f for f, _ in fields.values()],
                            offsets=[o for _, o in fields.values()], itemsize=C.sizeof(B)))
    base_params = np.frombuffer(bytes(N.default_params()), dtype=np.dtype(N.Params))[0]
    stat_names = np.dtype(N.Stats).names

    def solve_many(problems: list) -> list:
        n = len(problems)
        items = (B * n)()
        a = np.frombuffer(items, dtype=item_dt) if n else np.zeros(0, item_dt)
        a["params"] = base_params
        prm = a["params"]
        keep = []
        cols = {k: [] for k in ("solver", "f0", "n0", "f1", "n1", "mask0_out", "mask1_out", "t0", "t1", "scw",
                                "min_it", "max_it", "lo", "seed", "conf")}
        grids = []
        for j, pr in enumerate(problems):
            kind = pr["kind"]
            cols["solver"].append(_SOLVERS[kind])
            if kind == "sift":
                f0, f1 = pr["scale_features"], pr["orientation_features"]
                t0, t1 = pr["scale_residual_thresh"], pr["orientation_residual_thresh"]
            elif kind in ("homography", "fundamental"):
                f0, f1, t0, t1 = pr["correspondences"], None, pr["threshold"], 2.0
            else:
                f0, f1, t0, t1 = pr["features"], None, pr["scale_residual_thresh"], 2.0
            f0 = np.ascontiguousarray(f0, dtype=np.float64)
            f1 = None if f1 is None else np.ascontiguousarray(f1, dtype=np.float64)
            m0 = np.zeros(f0.shape[0], dtype=np.uint8)
            m1 = None if f1 is None else np.zeros(f1.shape[0], dtype=np.uint8)
            keep.append((f0, f1, m0, m1))
            cols["f0"].append(f0.ctypes.data)
            cols["n0"].append(f0.shape[0])
            cols["f1"].append(f1.ctypes.data if f1 is not None else 0)
            cols["n1"].append(f1.shape[0] if f1 is not None else 0)
            cols["mask0_out"].append(m0.ctypes.data)
            cols["mask1_out"].append(m1.ctypes.data if m1 is not None else 0)
            st = problem_settings(pr)
            cols["t0"].append(float(t0))
            cols["t1"].append(float(t1))
            cols["scw"].append(float(st["spatial_coherence_weight"]))
            cols["min_it"].append(int(st["min_iteration_number"]))
            cols["max_it"].append(int(st["max_iteration_number"]))
            cols["lo"].append(int(st["max_local_optimization_number"]))
            cols["seed"].append(int(st["seed"]))
            cols["conf"].append(float(st["confidence"]))
            if kind in ("homography", "fundamental"):
                grids.append((j, P.grid_params(f0, *st["image_sizes"], st["neighborhood_size"], from_data=False)))
        if n:
            for k in ("solver", "f0", "n0", "f1", "n1", "mask0_out", "mask1_out"):
                a[k] = cols[k]
            for k, name in (("t0", "scale_residual_thresh"), ("t1", "orientation_residual_thresh"),
                            ("scw", "spatial_coherence_weight"), ("min_it", "min_iteration_number"),
                            ("max_it", "max_iteration_number"), ("lo", "max_local_optimization_number"),
                            ("seed", "seed"), ("conf", "confidence")):
                prm[name] = cols[k]
            for j, (cells, sizes) in grids:
                prm["cell_number"][j] = cells
                if cells:
                    prm["cell_size"][j] = sizes
        N.check(N.lib.gcr_solve_batch(device, items, n, concurrency))
        out = []
        if not n:
            return out
        results = a["result"].tolist()
        Hs = a["H_out"].copy()
        stats = a["stats_out"].tolist()
        for j, (r, (f0, f1, m0, m1)) in enumerate(zip(results, keep)):
            masks = (m0.view(bool),) if m1 is None else (m0.view(bool), m1.view(bool))
            H = Hs[j].reshape(3, 3) if r > 0 else None
            out.append(dict(H=H, model=items[j].model_out if cols["solver"][j] < 3 and r > 0 else None,
                            num_inliers=r, stats=dict(zip(stat_names, stats[j])), masks=masks))
        return out

    return solve_many
