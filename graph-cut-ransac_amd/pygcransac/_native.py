"""ctypes view of the engine's C ABI (include/gcr.h).

The shared library ``libgcr.so`` is built in-tree next to this file (see
``graph-cut-ransac_amd/csrc/Makefile``).  Importing this module fails loudly if
it is missing: there is no CPU fallback for the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# GCR_LIB selects an alternative in-tree build of the same engine (the
# diagnostic libgcr_stamps.so of tools/stamp_probe.py)
LIB_PATH = os.path.join(_HERE, os.environ.get("GCR_LIB", "libgcr.so"))

GCR_OK = 0
GCR_EINVAL = -22
GCR_ENODEV = -19
SOLVER_SCALE3, SOLVER_SCALE3_ORIGINAL, SOLVER_SIFT22, SOLVER_HOMOGRAPHY4, SOLVER_FUNDAMENTAL7 = 0, 1, 2, 3, 4
FLAG_NO_LO = 1


class Params(C.Structure):
    _fields_ = [
        ("scale_residual_thresh", C.c_double),
        ("orientation_residual_thresh", C.c_double),
        ("spatial_coherence_weight", C.c_double),
        ("min_iteration_number", C.c_uint64),
        ("max_iteration_number", C.c_uint64),
        ("max_local_optimization_number", C.c_uint64),
        ("confidence", C.c_double),
        ("seed", C.c_uint64),
        ("batch_slots", C.c_uint32),
        ("flags", C.c_uint32),
        ("cell_size", C.c_double * 4),      # H / F neighbourhood grid (x1, y1, x2, y2)
        ("cell_number", C.c_uint32),        # cells along every axis, 0 = empty grid
        ("reserved", C.c_uint32),
    ]


class RectModel(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("x0", "y0", "s", "h7", "h8", "alpha", "phi")]


class Stats(C.Structure):
    _fields_ = [
        ("iteration_number", C.c_uint64),
        ("local_optimization_number", C.c_uint64),
        ("graph_cut_number", C.c_uint64),
        ("slots", C.c_uint64),
        ("hypotheses", C.c_uint64),
        ("hypotheses_computed", C.c_uint64),
        ("lo_models", C.c_uint64),
        ("launches", C.c_uint64),
        ("score", C.c_double),
        ("ms_setup", C.c_double),
        ("ms_generate", C.c_double),
        ("ms_score", C.c_double),
        ("ms_replay", C.c_double),
        ("ms_lo", C.c_double),
        ("ms_refit", C.c_double),
        ("ms_total", C.c_double),
        ("ms_score_kernel", C.c_double),
        ("ms_lo_lists", C.c_double),
        ("ms_lo_fit", C.c_double),
        ("ms_lo_score", C.c_double),
        ("ms_refit_fit", C.c_double),
        ("prefetched_chunks", C.c_uint64),
        ("exact_models", C.c_uint64),
        ("exact_pairs", C.c_uint64),
        ("exact_flips", C.c_uint64),
        ("ms_exact", C.c_double),
        ("near_ties", C.c_uint64),
        ("near_tie_flips", C.c_uint64),
        ("lo_refolds", C.c_uint64),
        ("chunk_msac_lists", C.c_uint64),
    ]

    def as_dict(self):
        # one read of the whole struct through a numpy record (ints and floats
        # as getattr would give them), not 30-odd ctypes attribute reads
        return dict(zip(_STATS_NAMES, np.frombuffer(self, dtype=_STATS_DT)[0].tolist()))


_STATS_DT = np.dtype(Stats)
_STATS_NAMES = _STATS_DT.names


class BatchResult(C.Structure):
    _fields_ = [
        ("models", C.c_uint64),
        ("iterations", C.c_uint64),
        ("best_slot", C.c_int64),
        ("best_score", C.c_double),
        ("best_inliers", C.c_uint64 * 2),
        ("best_model", RectModel),
    ]


class BatchItem(C.Structure):
    _fields_ = [
        ("solver", C.c_int),
        ("f0", C.POINTER(C.c_double)),
        ("n0", C.c_size_t),
        ("f1", C.POINTER(C.c_double)),
        ("n1", C.c_size_t),
        ("params", Params),
        ("mask0_out", C.POINTER(C.c_uint8)),
        ("mask1_out", C.POINTER(C.c_uint8)),
        ("H_out", C.c_double * 9),
        ("model_out", RectModel),
        ("stats_out", Stats),
        ("result", C.c_int),
    ]


# int (*)(void* user, const void* send, void* recv, size_t bytes)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"pygcransac: HIP engine library not found at {LIB_PATH}; build it with "
            "`make -C graph-cut-ransac_amd/csrc` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    dp, u8p, u32p = C.POINTER(C.c_double), C.POINTER(C.c_uint8), C.POINTER(C.c_uint32)
    vp = C.c_void_p
    L.gcr_last_error.restype = C.c_char_p
    L.gcr_abi_version.restype = C.c_int
    L.gcr_device_count.restype = C.c_int
    L.gcr_kernel_build_id.restype = C.c_char_p
    L.gcr_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.gcr_synchronize.argtypes = [vp]
    L.gcr_destroy.argtypes = [vp]
    L.gcr_destroy.restype = None
    L.gcr_default_params.argtypes = [C.POINTER(Params)]
    L.gcr_default_params.restype = None
    # the public entry points take their arrays as plain addresses (c_void_p
    # also accepts typed pointers): the wrappers pass ndarray.ctypes.data,
    # a third of their per-call Python cost otherwise
    L.gcr_rect_scale_only.argtypes = [vp, vp, C.c_size_t, C.POINTER(Params), C.c_int, vp, vp,
                                      C.POINTER(RectModel), C.POINTER(Stats)]
    L.gcr_rect_sift.argtypes = [vp, vp, C.c_size_t, vp, C.c_size_t, C.POINTER(Params), vp, vp, vp,
                                C.POINTER(RectModel), C.POINTER(Stats)]
    L.gcr_problem_create.argtypes = [vp, C.c_int, dp, C.c_size_t, dp, C.c_size_t, C.POINTER(vp)]
    L.gcr_problem_destroy.argtypes = [vp]
    L.gcr_problem_destroy.restype = None
    L.gcr_problem_run.argtypes = [vp, C.POINTER(Params), u8p, u8p, dp, C.POINTER(RectModel), C.POINTER(Stats)]
    L.gcr_problem_run_sharded.argtypes = [vp, C.POINTER(Params), C.c_int, C.c_int, ALLGATHER_FN, vp, u8p, u8p, dp,
                                          C.POINTER(RectModel), C.POINTER(Stats)]
    L.gcr_comm_unique_id.argtypes = [u8p]
    L.gcr_comm_create.argtypes = [vp, C.c_int, C.c_int, u8p, C.POINTER(vp)]
    L.gcr_comm_destroy.argtypes = [vp]
    L.gcr_comm_destroy.restype = None
    L.gcr_problem_run_comm.argtypes = [vp, C.POINTER(Params), vp, u8p, u8p, dp, C.POINTER(RectModel),
                                       C.POINTER(Stats)]
    L.gcr_solve_batch.argtypes = [C.c_int, C.POINTER(BatchItem), C.c_size_t, C.c_int]
    L.gcr_problem_verify_batch.argtypes = [vp, C.POINTER(Params), C.c_uint64, C.c_uint32, C.POINTER(BatchResult),
                                           C.POINTER(Stats)]
    L.gcr_problem_verify_batches.argtypes = [vp, C.POINTER(Params), C.c_uint64, C.c_uint32, C.c_uint32,
                                             C.POINTER(BatchResult), C.POINTER(Stats)]
    L.gcr_debug_generate.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_uint32, u8p, C.POINTER(RectModel)]
    L.gcr_debug_score.argtypes = [vp, C.POINTER(Params), C.POINTER(RectModel), C.c_uint32, u32p, u32p, dp, dp, dp]
    L.gcr_debug_score_less.argtypes = [vp, C.POINTER(Params), C.POINTER(RectModel), C.POINTER(RectModel)]
    L.gcr_debug_exchange_log.argtypes = [C.POINTER(C.c_uint64), C.c_size_t]
    L.gcr_debug_exchange_log.restype = C.c_size_t
    L.gcr_debug_mask.argtypes = [vp, C.POINTER(Params), C.POINTER(RectModel), C.c_int, C.c_int, u8p]
    L.gcr_host_log.argtypes = [C.c_double]
    L.gcr_host_log.restype = C.c_double
    L.gcr_host_pow_m3.argtypes = [C.c_double]
    L.gcr_host_pow_m3.restype = C.c_double
    L.gcr_host_atan2.argtypes = [C.c_double, C.c_double]
    L.gcr_host_atan2.restype = C.c_double
    L.gcr_host_math.argtypes = [C.c_int, C.c_double, C.c_double]
    L.gcr_host_math.restype = C.c_double
    L.gcr_host_sample.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                  C.c_uint32, u32p]
    L.gcr_debug_math.argtypes = [vp, C.c_int, dp, dp, C.c_size_t, dp]
    L.gcr_measure_hbm.argtypes = [vp, C.c_size_t, C.c_int, dp]
    L.gcr_warp_perspective.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, dp, C.c_int, dp, vp, C.c_int,
                                       C.c_int]
    L.gcr_host_fit_nonminimal.argtypes = [C.c_int, dp, C.c_size_t, dp, C.c_size_t, u32p, C.c_size_t, u32p,
                                          C.c_size_t, C.POINTER(RectModel)]
    L.gcr_debug_fit_nonminimal.argtypes = [vp, u32p, C.c_size_t, u32p, C.c_size_t, C.c_int, C.POINTER(RectModel)]
    L.gcr_find_homography.argtypes = [vp, vp, C.c_size_t, C.POINTER(Params), vp, vp, C.POINTER(Stats)]
    L.gcr_debug_generate_h.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_uint32, u8p, dp]
    L.gcr_debug_score_h.argtypes = [vp, C.POINTER(Params), dp, C.c_uint32, u32p, dp, dp]
    L.gcr_debug_mask_h.argtypes = [vp, C.POINTER(Params), dp, C.c_int, u8p]
    L.gcr_host_fit_h.argtypes = [dp, C.c_size_t, u32p, C.c_size_t, dp]
    L.gcr_find_fundamental_matrix.argtypes = L.gcr_find_homography.argtypes
    L.gcr_host_fit_f.argtypes = L.gcr_host_fit_h.argtypes
    L.gcr_host_grid_edges.argtypes = [dp, C.c_size_t, C.c_int, dp, C.c_uint64, u32p, C.c_size_t,
                                      C.POINTER(C.c_size_t)]
    L.gcr_host_bk_energy.argtypes = [C.c_size_t, dp, u32p, dp, C.c_size_t, u8p]
    L.gcr_host_labeling.argtypes = [dp, C.c_size_t, C.c_double, C.c_double, dp, C.c_int, dp, C.c_uint64, u8p]
    L.gcr_host_weighted_mode.argtypes = [dp, dp, C.c_size_t, C.c_double]
    L.gcr_host_weighted_mode.restype = C.c_double
    L.gcr_host_homography.argtypes = [C.POINTER(RectModel), dp]
    L.gcr_host_homography.restype = None
    L.gcr_host_residuals.argtypes = [C.c_int, C.c_int, dp, C.c_size_t, C.POINTER(RectModel), C.c_int, dp]
    L.gcr_host_residuals.restype = C.c_int
    return L


lib = _load()

_ctx_lock = threading.Lock()
_contexts: dict[int, int] = {}


def default_device() -> int:
    for var in ("GCR_DEVICE", "LOCAL_RANK"):
        if var in os.environ:
            try:
                return int(os.environ[var])
            except ValueError:
                pass
    return 0


def context(device: int | None = None) -> int:
    """Per-device engine context (created lazily, kept for the process)."""
    dev = default_device() if device is None else int(device)
    with _ctx_lock:
        h = _contexts.get(dev)
        if h is None:
            out = C.c_void_p()
            rc = lib.gcr_create(dev, C.byref(out))
            check(rc)
            h = out.value
            _contexts[dev] = h
        return h


def last_error() -> str:
    msg = lib.gcr_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc: int) -> int:
    if rc >= 0:
        return rc
    msg = last_error() or f"engine error {rc}"
    if rc == GCR_EINVAL:
        raise ValueError(msg)
    raise RuntimeError(msg)


def default_params() -> Params:
    p = Params()
    lib.gcr_default_params(C.byref(p))
    return p


def exchange_log():
    """The collective events of the calling thread's last summary replay
    (GCR_EXCHANGE_LOG=1; gcr_debug_exchange_log): a list of (kind, chunk,
    flags, arg) tuples -- kind 1 chunk issue (flags: set | ahead << 1, arg:
    slots), 2 re-summary (flags: set | locate << 1, arg: owner + 1 | from_pos
    << 16), 3 chunk collected."""
    n = lib.gcr_debug_exchange_log(None, 0)
    buf = (C.c_uint64 * max(n, 1))()
    lib.gcr_debug_exchange_log(buf, n)
    w = list(buf)[:n]
    return [tuple(w[i:i + 4]) for i in range(0, n, 4)]
