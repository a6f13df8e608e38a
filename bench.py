#!/usr/bin/env python3
"""bench.py -- hypotheses/s of the hypothesize-and-verify hot path on MI355X.

Metric (BASELINE.json): "model hypotheses/sec + wall-time to 0.99 confidence,
N=10k corrs 50% outliers".  Workload (BASELINE.json configs[1], the hybrid
rectification path on one MI355X): synthetic M2 problem,
N_s = 5000 scale + N_o = 5000 orientation features, 50 % outliers each, fp64.

One step = one pass of the hot path over one batch: `--slots` (default 4096,
configs[1]) outer-iteration slots are drawn (Philox), validated and solved,
every resulting model is MSAC-scored against all 10 000 features, and the
batch's first strict best (the reference's update rule, GCRANSAC.h:440-446) is
selected -- all on the device: one fused kernel (k_score_fm<..., true>:
in-kernel generation, exact MSAC sums, per-workgroup best) plus k_select_wg.
The correspondence workloads (h, f) generate in their own kernel and are
pipelined over two streams (batch b + 1 generated while batch b is scored).
The K timed steps are queued back to back (gcr_problem_verify_batches; for the
rectification workloads consecutive fused launches alternate between two HIP
streams, so one launch's workgroups take the CUs the other's early finishers
free -- GCR_VERIFY_OVERLAP=0 keeps them on one stream) and bracketed by device
synchronisation.  Features are uploaded once before
timing (HBM-resident).  `value` is the whole-job hypotheses/s; the end-to-end
latency of a full estimator call at confidence 0.99 (including LO and the
final refit) is reported beside it.

Multi-GPU: one process per GPU.  `--gpus N` without a launcher's WORLD_SIZE
spawns the N ranks itself (fresh child processes with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* set, started before this process touches HIP); under
torchrun the ranks come from the environment.  `--mode weak` (default): each
rank solves its own image pair (no data-path collective) and the final per-rank
best models are gathered with one RCCL all_gather.  `--mode strong`: ONE
N = 10 000 problem with a fixed hypothesis budget, every chunk of slots split
over the ranks and all-gathered (gcr_problem_run_sharded, SURVEY.md §8(e)
row 2), so the metric has a 1/2/4/8-GPU form on a single problem.
"""
import argparse
import ctypes as C
import json
import os
import socket
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "graph-cut-ransac_amd"))

METRIC = "model hypotheses/sec + wall-time to 0.99 confidence, N=10k corrs 50% outliers"
HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X vector fp64 spec
N_SIMD = 256 * 4               # CUs x SIMDs
CLOCK_GHZ = 2.4                # MI355X peak engine clock (spec)
# VALU issue costs, NANOSECONDS per wave64 instruction per SIMD, measured by
# tools/micro/valu_issue.hip on MI355X (profiles/r5_valu_issue.log): 16
# independent chains per wave, 4 waves per SIMD, each SIMD's cost = the span
# of its own waves (first start to last end, s_memrealtime, SIMDs told apart
# by HW_ID / XCC_ID) over the instructions they issued.  Round 4's per-wave
# figure (3.03 "cycles" for f64) assumed the 4 waves of a SIMD overlap for
# their whole run; their spans show they do not (4.4 s_memtime cycles per f64
# instruction at the measured ~2.3 GHz, against the spec's 4).  Priced without
# any clock assumption.  Classes = the SQ_INSTS_VALU_* counters; MUL_F32 is
# taken as ADD_F32.
VALU_CLASS_NS = {
    "SQ_INSTS_VALU_ADD_F32": 1.193, "SQ_INSTS_VALU_MUL_F32": 1.193, "SQ_INSTS_VALU_FMA_F32": 1.738,
    "SQ_INSTS_VALU_TRANS_F32": 3.470,
    "SQ_INSTS_VALU_ADD_F64": 1.885, "SQ_INSTS_VALU_MUL_F64": 1.916, "SQ_INSTS_VALU_FMA_F64": 1.967,
    "SQ_INSTS_VALU_TRANS_F64": 6.813,
    "SQ_INSTS_VALU_INT32": 1.199, "SQ_INSTS_VALU_INT64": 1.987, "SQ_INSTS_VALU_CVT": 1.860,
}
# the "other" bucket, per opcode (same micro-benchmark); v_cndmask_b32 at its
# SGPR-mask form (the VCC form's 8.0 ns alone is a back-to-back VCC-read
# penalty: 2.0 ns inside an instruction stream); the compare and readlane
# loops also issue the consumers of their SGPR results (two v_xor_b32 per
# compare, one v_add_u32 per readlane: tools/isa_loops.py on the micro's
# code), which are taken off (compare 4.897 / 6.017 - 2 x 1.208, readlane
# 3.803 - 1.199); unlisted 32-bit ops at the v_xor_b32 cost, unlisted 64-bit
# ops at the v_max_f64 cost
VALU_OP_NS = {
    "v_mov_b32": 1.039, "v_mov_b64": 1.834, "v_cndmask_b32": 1.931, "v_xor_b32": 1.208,
    "v_writelane_b32": 1.848, "v_readlane_b32": 2.604, "v_readfirstlane_b32": 2.604,
    "v_mbcnt_lo_u32_b32": 1.841, "v_mbcnt_hi_u32_b32": 1.841, "v_max_f64": 1.878, "v_min_f64": 1.878,
    "v_ldexp_f64": 1.955, "v_fract_f64": 1.929, "v_div_scale_f64": 1.860, "v_div_fmas_f64": 1.826,
    "v_div_fixup_f64": 1.839, "v_cmp_int": 2.481, "v_cmp_f64": 3.601,
}
# the model checked on a known mix (the micro-benchmark's MIX kernel: 3 f64
# add, 2 mul, 1 fma, 2 u32 add, 2 cndmask, 1 mov, 1 xor per iteration):
# predicted 20.155 ns against 19.241 measured per iteration per SIMD
VALU_MODEL_CHECK = {"mix_predicted_ns": 20.155, "mix_measured_ns": 19.241, "residual": 20.155 / 19.241 - 1.0,
                    "source": "profiles/r5_valu_issue.log (tools/micro/valu_issue.hip)"}


def op_ns(op):
    """issue cost of one other-bucket VALU opcode (llvm-objdump mnemonic)"""
    o = op.split("_e32")[0].split("_e64")[0].split("_sdwa")[0].split("_dpp")[0]
    if o.startswith(("v_cmp", "v_cmpx")):
        return VALU_OP_NS["v_cmp_f64"] if "f64" in o else VALU_OP_NS["v_cmp_int"]
    if o in VALU_OP_NS:
        return VALU_OP_NS[o]
    return VALU_OP_NS["v_max_f64"] if "f64" in o or "b64" in o or "64" in o else VALU_OP_NS["v_xor_b32"]


def other_split(pmc, mix):
    """The other bucket's executed opcode counts: each region's execution count
    of profiles/valu_mix.json (tools/valu_mix.py: loops of the kernel's code,
    their static per-class counts and other-opcode histograms) fitted by
    non-negative least squares to the PMC per-class counts and total, then the
    regions' other histograms weighted by them.  Returns (counts, fit residual)
    or None."""
    try:
        import numpy as np
        from scipy.optimize import nnls
    except ImportError:
        return None
    classes = [k.replace("SQ_INSTS_VALU_", "") for k in VALU_CLASS_NS]
    groups = {}
    for g in mix["regions"]:                      # identical regions (unrolled copies) fit as one
        key = json.dumps([g["classes"], g["other"]], sort_keys=True)
        groups.setdefault(key, g)
    regs = list(groups.values())
    rows = [[g["classes"].get(c, 0) for g in regs] for c in classes] + [[g["valu"] for g in regs]]
    rhs = [pmc.get("SQ_INSTS_VALU_" + c, 0.0) for c in classes] + [pmc["SQ_INSTS_VALU"]]
    A, b = np.array(rows, float), np.array(rhs, float)
    sc = 1.0 / np.maximum(b, 1e3)
    w, _ = nnls(A * sc[:, None], b * sc)
    pred = A @ w
    counts = {}
    for g, wi in zip(regs, w):
        for op, n in g["other"].items():
            counts[op] = counts.get(op, 0.0) + n * wi
    other_pmc = pmc["SQ_INSTS_VALU"] - sum(pmc.get(k, 0.0) for k in VALU_CLASS_NS)
    fit = {"max_class_rel_err": float(max(abs(p - q) / max(q, 1.0) for p, q in zip(pred[:-1], b[:-1])
                                          if q > 0.001 * b[-1])),
           "other_fit": float(sum(counts.values())), "other_pmc": float(other_pmc), "regions": len(regs)}
    return counts, fit


def valu_issue_ns(pmc, mix=None):
    """SIMD-nanoseconds of issue of one launch's VALU instructions, summed over
    the SIMDs: per-class counts x VALU_CLASS_NS, the other bucket split by
    opcode (other_split) and priced per opcode (op_ns) -- or, without a
    matching valu_mix entry, at the v_xor_b32 cost.  None unless every class
    counter was collected."""
    if not pmc or not pmc.get("SQ_INSTS_VALU") or any(k not in pmc for k in VALU_CLASS_NS):
        return None
    classed = sum(pmc[k] for k in VALU_CLASS_NS)
    other = max(0.0, pmc["SQ_INSTS_VALU"] - classed)
    ns = sum(pmc[k] * c for k, c in VALU_CLASS_NS.items())
    split = other_split(pmc, mix) if mix else None
    info = {"per_class_insts": {k.replace("SQ_INSTS_VALU_", ""): pmc[k] for k in VALU_CLASS_NS},
            "other_insts": other}
    if split:
        counts, fit = split
        tot = sum(counts.values()) or 1.0
        # the fitted mix's average cost, applied to the measured other count
        avg = sum(n * op_ns(op) for op, n in counts.items()) / tot
        ns += other * avg
        top = sorted(counts.items(), key=lambda kv: -kv[1])[:12]
        info.update({"other_avg_ns": avg, "other_split_fit": fit,
                     "other_top_share": {op: n / tot for op, n in top}})
    else:
        ns += other * VALU_OP_NS["v_xor_b32"]
        info["other_avg_ns"] = VALU_OP_NS["v_xor_b32"]
    return ns, info


def valu_mix_entry(kernel, build_id):
    """profiles/valu_mix.json's entry for `kernel` of this kernel build, or None"""
    path = os.path.join(REPO, "profiles", "valu_mix.json")
    try:
        with open(path) as f:
            ent = json.load(f).get(kernel)
    except (OSError, ValueError):
        return None
    if ent is None or ent.get("kernel_build_id") != build_id:
        return None
    return ent


def score_kernel_name(kind, slots):
    """The fused generate+score instantiation launch_verify_fused picks
    (kernels.hip split_h); the bench's step launches it plus k_select_wg."""
    h = int(os.environ.get("GCR_SPLIT_H", "0") or 0)
    # the fundamental matrix scores up to 3 models per slot (launch size 3 x slots)
    nh = slots * 3 if kind == 4 else slots
    if h not in (64, 16, 4):
        h = 64 if nh >= 16384 else 16 if nh >= 2048 else 4
    # the correspondence paths generate in k_generate<3, G> / k_generate_f<G>
    # and score unfused
    fused = "false" if kind >= 3 else "true"
    # H = 16 launches use the feature-major scorer unless GCR_SCORER=split
    # (kernels.hip use_fm); so do correspondence launches of >= 16384
    # hypotheses unless GCR_GEO_FM_LARGE=0 (kernels.hip launch_score_geo)
    fm = not os.environ.get("GCR_SCORER", "").startswith("s")
    if h == 16 and fm:
        return f"k_score_fm<{kind}, 16, {fused}>"
    if h == 64 and kind >= 3 and fm and os.environ.get("GCR_GEO_FM_LARGE", "1") != "0":
        return f"k_score_fm<{kind}, 16, {fused}>"
    return f"k_score_split<{kind}, {h}, {dict([(64, 120), (16, 420), (4, 960)])[h]}, {fused}>"


def traffic_per_launch(ent):
    """HBM bytes per launch from a PMC entry (profiles/pmc_traffic.json, written
    by tools/pmc_summary.py from separate --pmc passes: 2 x FETCH_SIZE +
    WRITE_SIZE per dispatch, the gfx950 correction of MI355X_MICROARCH.md);
    None if this kernel/batch/build was not profiled."""
    return None if ent is None else ent.get("hbm_bytes_per_launch")


def pmc_entry(kernel, slots, build_id=None):
    """The committed PMC summary of `kernel` at this batch size, or None.  An
    entry counts only if it was collected from the kernels this process runs:
    its `kernel_build_id` (tools/pmc_summary.py) must equal the loaded
    library's gcr_kernel_build_id() (SHA-256 of the kernels' sources and
    flags); counters of an older build are never reused."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            table = json.load(f)
    except (OSError, ValueError):
        return None
    ent = table.get(f"{kernel}@{slots}")
    if ent is None or build_id is None or ent.get("kernel_build_id") != build_id:
        return None
    return ent


# The fundamental matrix yields 1-3 models per 7-point sample (≈1.07 live per
# slot at the F config), and the batch scorer runs one workgroup of 16 live
# hypotheses per CU.  Rounds 2-4 used 3712 slots (≈3970 live models, one wave
# of workgroups).  Since round 5 the large correspondence launches use the
# same feature-major scorer (k_compact first), and the generator -- latency-
# bound at ~1 wave per SIMD -- hides more of its latency in bigger launches:
# 3712 / 7424 / 11136 / 14848 / 22272 / 29696 slots -> 3.21 / 3.65 / 3.94 /
# 4.25 / 4.25 / 4.22 x 10^7 hypotheses/s (two-stream pipeline, one box).
F_SLOTS = 14848
# full estimator calls timed for the 0.99-confidence wall time (seeds 100..);
# the number of graph-cut rounds, hence the time, varies with the seed
# (1.3-3.1 ms for M2), so the median is taken over 11 calls
LAT_CALLS = 11
# untimed warm-up floor: the driver's short runs (--warmup 5 = 0.7 ms) would
# otherwise time the clock ramp; extra warm-up batches run at slots past the
# timed region until this much wall time has passed (reported, not counted)
WARMUP_FLOOR_MS = 200.0
# the box's CPU share for one GPU (gpurun: 16 host threads per GPU)
CPU_SHARE = 16


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--workload", choices=["m2", "m1", "h", "f", "batch"], default="m2",
                    help="m2: configs[1] hybrid rectification (headline); m1: scale-only; "
                         "h: configs[2] 4-pt homography, N=5000, 50%% outliers; "
                         "f: configs[3] 7-pt fundamental matrix, N=10000, 80%% outliers; "
                         "batch: configs[4] mixed H / F / rectification problems, full estimator calls")
    ap.add_argument("--problems", type=int, default=1024, help="batch workload: problems in the whole job")
    ap.add_argument("--concurrency", type=int, default=12, help="batch workload: host threads per GPU")
    ap.add_argument("--batch-lambda", type=float, default=None,
                    help="batch workload: spatial_coherence_weight of the H / F problems (default: the entry "
                         "points' 0.975, graph-cut LO with pairwise terms; 0 isolates the graph-cut share)")
    ap.add_argument("--slots", type=int, default=None,
                    help="outer-iteration slots per launch (default 4096; f: 14848, see F_SLOTS)")
    ap.add_argument("--mode", choices=["weak", "strong"], default="weak",
                    help="weak: one problem per rank (default); strong: one problem, every chunk of slots "
                         "sharded over the ranks (budget = steps x slots, default 65536 slots per step)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget per leg (0 = skip)")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-hbm-probe", action="store_true", help="skip the measured-HBM-peak copy probe")
    return ap.parse_args(argv)


# ------------------------------------------------------------ rank launcher ---
def rank_env(base, rank, world, port, addr="127.0.0.1"):
    """Environment of rank `rank` of a `world`-rank job on this node (what
    torchrun would set): one process per GPU, LOCAL_RANK selects the device."""
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR=addr, MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")      # dmabuf IPC only on these hosts
    return env


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv, world, script=None):
    """Start `world` fresh bench processes (this file, same arguments) and wait
    for them.  Rank 0 writes the JSON line to our stdout; the other ranks'
    stdout goes to stderr.  Called before anything here touches HIP.  Returns
    the first non-zero exit status (the remaining ranks are then terminated),
    else 0."""
    port = free_port()
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__), *argv],
                                      env=rank_env(os.environ, r, world, port),
                                      stdout=None if r == 0 else sys.stderr))
    rc = 0
    while procs and rc == 0:
        for p in list(procs):
            code = p.poll()
            if code is not None:
                procs.remove(p)
                if code != 0:
                    rc = code if code > 0 else 128 - code
        time.sleep(0.05)
    for p in procs:                          # a rank failed: stop the others
        p.terminate()
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    return rc


def workload_problem(name, seed):
    """(f0, f1, thr0, thr1, solver, text) of a bench workload (solver = the
    engine's solver id: 0 scale-only, 2 hybrid, 3 homography, 4 fundamental).
    Pure numpy: nothing here touches the GPU."""
    from pygcransac import synthetic as S

    if name == "m2":
        f0, f1, _, _, thr0, thr1 = S.problem_m2(5000, 5000, seed=seed)
        return f0, f1, thr0, thr1, 2, ("M2 hybrid 2+2-SIFT rectification (findRectifyingHomographySIFT), "
                                       "5000 scale + 5000 orientation")
    if name == "h":
        f0, _, _, thr0 = S.problem_h(5000, 0.5, seed=seed)
        return f0, None, thr0, 0.0, 3, "H 4-point homography (findHomography), 5000 correspondences"
    if name == "f":
        f0, _, _, thr0 = S.problem_f(10_000, 0.8, seed=seed)
        return f0, None, thr0, 0.0, 4, "F 7-point fundamental matrix (findFundamentalMatrix), 10000 correspondences"
    f0, _, thr0 = S.problem_m1(10_000, seed=seed)
    return f0, None, thr0, 0.0, 0, "M1 3-SIFT scale-only rectification (findRectifyingHomographyScaleOnly), 10000 scale"


def host_cpu_info():
    """CPU model, usable cores and frequency governor of this host."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    gov = "unknown"
    try:
        with open("/sys/devices/system/cpu/cpu0/cpufreq/scaling_governor") as f:
            gov = f.read().strip()
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return dict(model=model, governor=gov, usable_cores=usable)


def _cpu_leg(a):
    """One CPU worker: the oracle's single-thread hot path over its slot range."""
    kind, f0, f1, thr0, thr1, seed, slot0, nslots, smp = a
    import oracle_ffi as O

    n, sec, _ = O.hot_batch(kind, f0, f1, thr0, thr1, seed, slot0, nslots, sampler=smp)
    return n, sec


def cpu_baseline(args):
    """The CPU oracle (tests/oracle_ffi, -O3, glibc math) on this host's cores:
    (1) one thread, as the reference runs; (2) P = min(CPU share, usable
    cores) independent worker processes on disjoint slot ranges of the same
    problem (throughput).  A bounded sample of about `--cpu-seconds` per leg.
    Also times the same full estimator call to 0.99 confidence (one run; not
    for F at 80 % outliers, ~490k iterations).  Runs before the GPU is
    touched; the workers are forked from this still GPU-free process."""
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi as O

    f0, f1, thr0, thr1, kind, _ = workload_problem(args.workload, 20251121)
    seed = 20251121
    # rectification: the reference's own sampler (random_device + mt19937 +
    # shuffle); H / F (no reference, finding 0.1): the cheaper Philox draw,
    # i.e. the stronger CPU baseline
    smp = O.SAMPLER_PHILOX if kind >= 3 else O.SAMPLER_FAITHFUL
    smp_text = "Philox counter sampler" if kind >= 3 else "reference-faithful random_device+mt19937+shuffle sampler"
    n_cal, s_cal, _ = O.hot_batch(kind, f0, f1, thr0, thr1, seed, 0, 64, sampler=smp)
    rate = n_cal / max(s_cal, 1e-6)
    nslots = max(64, int(64 * args.cpu_seconds / max(s_cal, 1e-6)))
    n1, s1 = _cpu_leg((kind, f0, f1, thr0, thr1, seed, 0, nslots, smp))
    info = host_cpu_info()
    P = max(1, min(CPU_SHARE, info["usable_cores"]))
    legs = [(kind, f0, f1, thr0, thr1, seed, (r + 1) * 10**8, nslots, smp) for r in range(P)]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(P) as pool:
        outs = pool.map(_cpu_leg, legs)
    wall = time.perf_counter() - t0
    nP = sum(n for n, _ in outs)
    cpu = dict(value=nP / wall, unit="hypotheses/s", cores=P, kind="port",
               sample=(f"{P} processes x {nslots} outer-iteration slots of the same workload (disjoint slot "
                       f"ranges), CPU oracle (glibc math, {smp_text}, g++ -O3), {wall:.1f} s wall"),
               single_thread=dict(value=n1 / s1, cores=1, seconds=s1, calibration_rate=rate),
               cpu=info)
    # the whole host (P = nproc).  The GPU box caps a one-GPU job
    # at its 16-thread CPU share, so the full-host figure is the measured
    # per-process rate of the P-process leg times the usable cores -- a
    # projection (perfect scaling, no turbo loss), labelled as such
    per_proc = nP / wall / P
    cpu["full_host"] = dict(value=per_proc * info["usable_cores"], cores=info["usable_cores"],
                            kind="projection", note=(f"{P}-process measured rate / {P} x {info['usable_cores']} "
                                                     "usable cores; not run (the box limits a one-GPU job to "
                                                     f"{CPU_SHARE} host threads)"))
    if not args.no_latency and kind != 4:
        t1 = time.perf_counter()
        kw = dict(min_it=0, max_it=10**7, lo=50, confidence=0.99, seed=100, math_mode=O.MATH_GLIBC, sampler=smp)
        if kind == 2:
            O.rect_sift(f0, f1, thr0, thr1, **kw)
        elif kind == 3:
            O.find_homography(f0, thr0, **kw)
        else:
            O.rect_scale_only(f0, thr0, **kw)
        cpu["oracle_call_ms"] = (time.perf_counter() - t1) * 1e3
        cpu["oracle_call_note"] = f"CPU oracle, 1 thread, glibc math, {smp_text}, same call (seed 100)"
    return cpu


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: spawn the ranks before this process loads the engine
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    if args.slots is None:
        args.slots = F_SLOTS if args.workload == "f" else 65536 if args.mode == "strong" else 4096
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0 and args.workload != "batch" and args.mode == "weak":
        cpu = cpu_baseline(args)               # host cores only, before the GPU is touched
    # "nccl" is RCCL on ROCm; GCR_DIST_BACKEND=gloo rehearses the multi-rank
    # path on fewer GPUs than ranks (host tensors, ranks share devices)
    backend = os.environ.get("GCR_DIST_BACKEND", "nccl")
    dist = None
    coll_dev = None
    from pygcransac import _native as N

    ndev = max(1, N.lib.gcr_device_count())
    device = local_rank % ndev
    if world > ndev and backend == "nccl":
        backend = "gloo"                       # RCCL needs one GPU per rank; rehearse on gloo
    if world > 1:
        import torch
        import torch.distributed as tdist

        if backend == "nccl":
            torch.cuda.set_device(device)
            coll_dev = torch.device("cuda", device)
        else:
            coll_dev = torch.device("cpu")
        tdist.init_process_group(backend)
        dist = tdist

    import numpy as np
    import pygcransac

    ctx = N.context(device)
    seed = 20251121 + rank
    if args.workload == "batch":
        return bench_batch(args, rank, world, dist, device, coll_dev)
    if args.mode == "strong":
        return bench_strong(args, rank, world, dist, device, coll_dev, backend)
    f0, f1, thr0, thr1, solver, workload = workload_problem(args.workload, seed)
    n_total = f0.shape[0] + (0 if f1 is None else f1.shape[0])
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    f0c = np.ascontiguousarray(f0)
    f1c = None if f1 is None else np.ascontiguousarray(f1)
    ph = C.c_void_p()
    N.check(N.lib.gcr_problem_create(ctx, solver, dp(f0c), f0c.shape[0], dp(f1c) if f1c is not None else None,
                                     0 if f1c is None else f1c.shape[0], C.byref(ph)))
    prob = ph.value
    p = N.default_params()
    p.scale_residual_thresh = thr0
    p.orientation_residual_thresh = thr1
    p.seed = seed

    rec_dt = np.dtype([("models", "<u8"), ("iterations", "<u8"), ("best_slot", "<i8"), ("best_score", "<f8"),
                       ("best_inliers", "<u8", 2), ("best_model", "<f8", 7)])
    assert rec_dt.itemsize == C.sizeof(N.BatchResult)

    def steps(k0, n):
        res = (N.BatchResult * n)()
        st = N.Stats()
        N.check(N.lib.gcr_problem_verify_batches(prob, C.byref(p), k0 * args.slots, args.slots, n, res,
                                                 C.byref(st)))
        return res, st

    def account(res, st, n, st_acc):
        # the batch records (already on the host when the call returns) are
        # read after the timed region: the host's bookkeeping is not the step
        if st_acc is not None:
            st_acc["kernel_ms"] += st.ms_score_kernel
            st_acc["launches"] += n
            rec = np.frombuffer(res, dtype=rec_dt, count=n)
            st_acc["models"] += int(rec["models"].sum())
            # first strict best over the batches, in slot order
            ok = (rec["best_slot"] >= 0) & (rec["best_score"] > st_acc["best_score"])
            if ok.any():
                sc = np.where(ok, rec["best_score"], -np.inf)
                i = int(np.argmax(sc))              # the first index of the maximum
                st_acc["best_score"] = float(rec["best_score"][i])
                bm = rec["best_model"][i]           # x0, y0, s, h7, h8, alpha, phi
                st_acc["best_model"] = (float(bm[3]), float(bm[4]), float(bm[5]), float(bm[6]))

    def barrier():
        N.check(N.lib.gcr_synchronize(ctx))
        if dist is not None:
            import torch

            if backend == "nccl":
                torch.cuda.synchronize()
            dist.barrier()

    t_w = time.perf_counter()
    if args.warmup:
        steps(0, args.warmup)
    N.check(N.lib.gcr_synchronize(ctx))
    extra, k_extra = 0, args.warmup + args.steps      # extra warm-up slots lie past the timed region
    while (time.perf_counter() - t_w) * 1e3 < WARMUP_FLOOR_MS:
        steps(k_extra + extra, 64)
        N.check(N.lib.gcr_synchronize(ctx))
        extra += 64
    warm_ms = (time.perf_counter() - t_w) * 1e3
    acc = dict(models=0, kernel_ms=0.0, launches=0, best_score=-1.0, best_model=(0.0, 0.0, 0.0, 0.0))
    barrier()
    t0 = time.perf_counter()
    timed = steps(args.warmup, args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    account(*timed, args.steps, acc)

    models_total = acc["models"]
    gathered = 1
    if dist is not None:
        import torch

        dev = coll_dev
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        m = torch.tensor([float(models_total)], dtype=torch.float64, device=dev)
        dist.all_reduce(m, op=dist.ReduceOp.SUM)
        models_total = int(m.item())
        # RCCL gather of the final per-rank models (the only collective)
        mine = torch.tensor([acc["best_score"], *acc["best_model"]], dtype=torch.float64, device=dev)
        outs = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(outs, mine)
        gathered = len(outs)

    value = models_total / elapsed
    kind = {N.SOLVER_SIFT22: 2, N.SOLVER_HOMOGRAPHY4: 3, N.SOLVER_FUNDAMENTAL7: 4}.get(solver, 0)
    kernel_name = score_kernel_name(kind, args.slots)
    avg_kernel_s = acc["kernel_ms"] / max(1, acc["launches"]) / 1e3
    models_per_launch = acc["models"] / max(1, acc["launches"])
    # algorithmic bytes per hypothesis: one pass over the feature SoA the
    # residual reads -- 3 doubles per rectification feature, 4 per
    # correspondence (x1, y1, x2, y2)
    bytes_per_feature = 32.0 if kind >= 3 else 24.0
    bytes_per_launch = models_per_launch * bytes_per_feature * n_total
    achieved = bytes_per_launch / avg_kernel_s / 1e9 if avg_kernel_s > 0 else 0.0

    # fp64 VALU view for the correspondence residuals (fixed work per pair):
    # homography transfer error 17 flops + 2 divisions, Sampson 32 + 1
    valu = None
    if kind >= 3 and avg_kernel_s > 0:
        flops_pair = 19.0 if kind == 3 else 33.0
        tf = models_per_launch * n_total * flops_pair / avg_kernel_s / 1e12
        valu = {"achieved_tflops": tf, "peak_tflops": FP64_VALU_PEAK_TFLOPS, "frac": tf / FP64_VALU_PEAK_TFLOPS,
                "flops_per_pair": flops_pair}
    # measured VALU occupancy of the dominant kernel from the committed PMC pass
    # (SQ_ACTIVE_INST_VALU counts quad-cycles): the fraction of the 1024 SIMDs'
    # cycles spent issuing VALU during one launch -- the bound the algorithmic
    # HBM figure above does not see (the features are L2-resident)
    build_id = N.lib.gcr_kernel_build_id().decode()
    pmc = pmc_entry(kernel_name, args.slots, build_id)
    if pmc and "SQ_ACTIVE_INST_VALU" in pmc and avg_kernel_s > 0:
        simd_cycles = N_SIMD * avg_kernel_s * CLOCK_GHZ * 1e9
        valu = dict(valu or {})
        valu.update({"active_frac": 4.0 * pmc["SQ_ACTIVE_INST_VALU"] / simd_cycles,
                     "insts_per_launch": pmc.get("SQ_INSTS_VALU"),
                     "lds_insts_per_launch": pmc.get("SQ_INSTS_LDS"),
                     "wait_frac": (pmc["SQ_WAIT_ANY"] / pmc["SQ_WAVE_CYCLES"]
                                   if pmc.get("SQ_WAVE_CYCLES") else None),
                     "clock_ghz": CLOCK_GHZ,
                     "source": "profiles/pmc_traffic.json (rocprofv3 --pmc, separate passes)"})

    # VALU issue bound of the dominant kernel: the committed PMC pass's VALU
    # instructions priced per class (and the other bucket per opcode) in
    # measured ns of one SIMD's issue, over what the 1024 SIMDs offer during
    # the live average launch
    valu_issue = None
    issue = None
    if pmc and pmc.get("SQ_INSTS_VALU") and avg_kernel_s > 0:
        valu_issue = {"insts_per_launch": pmc["SQ_INSTS_VALU"],
                      "wait_frac": (pmc["SQ_WAIT_ANY"] / pmc["SQ_WAVE_CYCLES"]
                                    if pmc.get("SQ_WAVE_CYCLES") and pmc.get("SQ_WAIT_ANY") else None),
                      "rocprof_avg_ms": pmc.get("rocprof_avg_ms"),
                      "source": f"profiles/pmc_traffic.json ({pmc.get('source')}, kernel build {build_id})"}
        issue = valu_issue_ns(pmc, valu_mix_entry(kernel_name, build_id))
        if issue is not None:
            ns, info = issue
            floor_s = ns * 1e-9 / N_SIMD
            valu_issue.update(info)
            valu_issue.update({"class_cost_ns": {k.replace("SQ_INSTS_VALU_", ""): c for k, c in VALU_CLASS_NS.items()},
                               "op_cost_ns": VALU_OP_NS, "model_check": VALU_MODEL_CHECK,
                               "issue_floor_ms": floor_s * 1e3, "frac": floor_s / avg_kernel_s})

    # wall time to 0.99 confidence: full estimator call (incl. upload, LO, refit)
    latency = None
    if not args.no_latency and rank == 0:
        lat, stats_all = [], []
        # r = -1: one untimed warm-up call (seed 99: the first call of a
        # process allocates the context's pinned LO / refit buffers, ~2 ms)
        for r in range(-1, LAT_CALLS):
            t1 = time.perf_counter()
            if solver == N.SOLVER_FUNDAMENTAL7:
                out = pygcransac.findFundamentalMatrix(f0, 960, 1280, 960, 1280, threshold=thr0, conf=0.99,
                                                       min_iters=0, max_iters=10**7, seed=100 + r, device=device,
                                                       return_stats=True)
            elif solver == N.SOLVER_HOMOGRAPHY4:
                out = pygcransac.findHomography(f0, 960, 1280, 960, 1280, threshold=thr0, conf=0.99,
                                                min_iters=0, max_iters=10**7, seed=100 + r, device=device,
                                                return_stats=True)
            elif solver == N.SOLVER_SIFT22:
                out = pygcransac.findRectifyingHomographySIFT(f0, f1, thr0, thr1, 0.0, 0, 10**7, 50, seed=100 + r,
                                                              confidence=0.99, device=device, return_stats=True)
            else:
                out = pygcransac.findRectifyingHomographyScaleOnly(f0, thr0, 0.0, 0, 10**7, 50, seed=100 + r,
                                                                   confidence=0.99, device=device,
                                                                   return_stats=True)
            if r < 0:
                continue
            lat.append((time.perf_counter() - t1) * 1e3)
            stats_all.append(out[-1])
        # the breakdown of the median call (LAT_CALLS is odd)
        last_stats = stats_all[sorted(range(len(lat)), key=lat.__getitem__)[len(lat) // 2]]
        latency = dict(ms_median=statistics.median(lat), ms_all=lat, warmup_calls=1,
                       iterations=last_stats["iteration_number"], hypotheses=last_stats["hypotheses"],
                       ms_breakdown={k: last_stats[k] for k in ("ms_setup", "ms_generate", "ms_score", "ms_replay",
                                                                "ms_lo", "ms_lo_lists", "ms_lo_fit", "ms_lo_score", "ms_refit_fit",
                                                                "ms_refit", "ms_total", "graph_cut_number")})

    if cpu is not None and latency is not None and "oracle_call_ms" in cpu:
        latency["cpu_oracle_ms"] = cpu.pop("oracle_call_ms")
        latency["cpu_oracle_note"] = cpu.pop("oracle_call_note")

    # the box's achievable HBM bandwidth (streaming copy), beside the spec peak
    hbm_meas = None
    if rank == 0 and not args.no_hbm_probe:
        g = C.c_double(0.0)
        if N.lib.gcr_measure_hbm(ctx, 2 << 30, 10, C.byref(g)) == 0 and g.value > 0:
            hbm_meas = g.value

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "hypotheses/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded M2/M1 generator, pygcransac/synthetic.py; notebook features absent)",
            "config": {
                "workload": workload,
                "n_features": n_total,
                "outlier_ratio": 0.8 if kind == 4 else 0.5,
                "hypotheses_per_launch": args.slots,
                "parallelism": f"problem-sharded x{world}" if world > 1 else "single GPU",
                "collective_backend": backend if world > 1 else None,
            },
            "roofline": {
                # the measured limiter: the features are L2-resident (traffic is
                # <1 % of the algorithmic bytes), so the ceiling that bounds the
                # dominant kernel is fp64 VALU issue, not HBM
                # null when no PMC pass of this kernel build exists
                "bound": "valu" if valu_issue and "frac" in valu_issue else None,
                # SIMDs kept busy issuing VALU (priced instructions, ns of issue
                # per second of the launch), against the 1024 SIMDs
                "achieved": (issue[0] * 1e-9 / avg_kernel_s if valu_issue and "frac" in valu_issue else None),
                "peak": N_SIMD,
                "unit": "SIMDs busy issuing VALU (measured per-instruction issue costs)",
                "frac": valu_issue.get("frac") if valu_issue else None,
                "traffic": traffic_per_launch(pmc),
                "valu_issue": valu_issue,
                "kernel": kernel_name,
                "kernel_build_id": build_id,
                "avg_kernel_ms": avg_kernel_s * 1e3,
                "avg_kernel_ms_note": ("HIP events on the engine's stream. Overlapped launches (rectification, "
                                       "two streams, GCR_VERIFY_OVERLAP): one event pair brackets the whole call "
                                       "and the per-launch time is that span over the launches -- the throughput "
                                       "time of one launch; a rocprofv3 dispatch lasts longer, since its "
                                       "workgroups also wait for CUs the other stream's launch holds "
                                       "(profiles/*_span.txt: first start to last end over the dispatches). "
                                       "One stream: when no deferred selection falls inside a call's launches "
                                       "1..K-2 (K <= 64), one event pair brackets those back-to-back launches "
                                       "and their mean is taken (GCR_TIMING_SPAN); otherwise pairs around every "
                                       "4th launch (GCR_TIMING_STRIDE), never the launch right after a "
                                       "deferred-selection flush. The mean is extrapolated to all launches. The "
                                       "whole queue, selections included, is ms_per_step"),
                "hypotheses_per_launch": models_per_launch,
                "algorithmic_hbm": {
                    "achieved_gbs": achieved,
                    "peak_gbs": HBM_PEAK_GBS,
                    "ratio": achieved / HBM_PEAK_GBS,
                    "measured_peak_gbs": hbm_meas,
                    "ratio_to_measured_peak": (achieved / hbm_meas) if hbm_meas else None,
                    "bytes_per_hypothesis": bytes_per_feature * n_total,
                    "note": ("ALGORITHMIC bytes (one pass over the feature rows per hypothesis, SURVEY §8(d)) / "
                             "the kernel's live average duration. NOT a roofline fraction: the features stay "
                             "L2/LDS-resident, so the ratio can exceed 1; real HBM bytes are `traffic`"),
                },
                "note": ("achieved/frac: the dominant kernel's VALU instructions per class "
                         "(SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_{F32,F64}, INT32, INT64, CVT; rocprofv3 --pmc passes of "
                         "this same kernel build, profiles/pmc_traffic.json) and the rest split by opcode "
                         "(profiles/valu_mix.json: the kernel's loops, their execution counts fitted to the class "
                         "counters) x their measured issue ns per SIMD (valu_issue.class_cost_ns / op_cost_ns, "
                         "tools/micro/valu_issue.hip per-SIMD spans; model checked on a known mix: "
                         "valu_issue.model_check) / the live average launch = SIMDs busy issuing, against 1024. "
                         "null when no PMC pass exists for this kernel build; the rest of the time is latency "
                         "(valu_issue.wait_frac)"),
            },
            "valu": valu,
            "cpu_baseline": cpu,
            "warmup_floor": {"ms": warm_ms, "extra_untimed_steps": extra,
                             "note": f"untimed warm-up runs until >= {WARMUP_FLOOR_MS:.0f} ms (clock ramp)"},
            "wall_time_to_0.99_confidence": latency,
            "gathered_models": gathered,
        }
        print(json.dumps(line))
    N.lib.gcr_problem_destroy(prob)
    if dist is not None:
        dist.barrier()          # rank 0's latency / CPU legs finish before teardown
        dist.destroy_process_group()


def bench_strong(args, rank, world, dist, device, coll_dev, backend):
    """Strong scaling on ONE problem: a fixed budget of
    steps x slots outer iterations of the workload, every fetched chunk of
    `--slots` slots split into `world` blocks, each rank generating and scoring
    its block on its own GPU, the per-hypothesis records all-gathered (RCCL on
    "nccl") and the replay / LO / refit run identically on every rank
    (gcr_problem_run_sharded), so every rank returns the single-rank result.
    value = the problem's scored hypotheses / the max-over-ranks wall time of
    the whole call (LO and refit included, they do not shard).  `--warmup W`
    runs the same call W times untimed first."""
    from pygcransac import _native as N
    from pygcransac import distributed as D

    seed = 20251121                            # the same problem on every rank
    f0, f1, thr0, thr1, solver, workload = workload_problem(args.workload, seed)
    budget = args.steps * args.slots
    coll = coll_dev if backend == "nccl" else None
    # RCCL: the engine's own communicator (ncclAllGather of the device block
    # summaries, no Python in the exchange); gloo: the callback exchange
    # (GCR_COMM=0: the callback on RCCL too)
    comm = None
    if backend == "nccl" and os.environ.get("GCR_COMM", "1") != "0":
        comm = D.Comm(dist, rank, world, device=device)

    def run(iters):
        prm = dict(scale_residual_thresh=thr0, orientation_residual_thresh=thr1, seed=seed,
                   min_iteration_number=iters, max_iteration_number=iters, batch_slots=args.slots)
        return D.run_problem_sharded(solver, f0, f1, prm, rank=rank, world=world, dist=dist, device=device,
                                     coll_device=coll, comm=comm)

    def barrier():
        N.check(N.lib.gcr_synchronize(N.context(device)))
        if dist is not None:
            dist.barrier()

    for _ in range(max(1, args.warmup)):                  # untimed warm-up: whole runs (their workspace
        run(budget)                                       # -- pinned buffers included -- is reused)
    barrier()
    t0 = time.perf_counter()
    _, masks, st, _ = run(budget)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        hyps = float(st["hypotheses"])
        verify_ms = st["ms_total"] - st["ms_lo"] - st["ms_refit"]
        print(json.dumps({
            "metric": METRIC,
            "value": hyps / elapsed,
            "unit": "hypotheses/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded generators, pygcransac/synthetic.py)",
            "config": {"workload": f"{workload}: one problem, fixed budget of {budget} outer iterations "
                                   f"({args.steps} chunks of {args.slots} slots), hypothesis-sharded",
                       "parallelism": f"hypothesis-sharded x{world} "
                                      f"({'gcr_problem_run_comm' if comm else 'gcr_problem_run_sharded'})",
                       "collective_backend": (("rccl-engine" if comm else backend) if world > 1 else
                                              ("rccl-engine" if comm else None)),
                       "iterations": st["iteration_number"], "hypotheses": st["hypotheses"],
                       "inliers": int(sum(int(m.sum()) for m in masks)),
                       "ms_breakdown": {k: st[k] for k in ("ms_setup", "ms_generate", "ms_score", "ms_replay",
                                                           "ms_lo", "ms_refit", "ms_total")},
                       "verify_phase_hypotheses_per_s": hyps / (verify_ms / 1e3) if verify_ms > 0 else None},
            "roofline": None,
            "cpu_baseline": None,
        }))
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def batch_problems(n, seed=20251121, lam=None):
    """BASELINE configs[4]: `n` independent problems, kinds cycling over
    homography / fundamental / hybrid rectification / scale-only, sizes
    U{1000 .. 10000}, 50 % outliers, confidence 0.99 (full estimator calls,
    LO and refit included)."""
    import numpy as np
    from pygcransac import synthetic as S

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        size = int(rng.integers(1000, 10001))
        k = i % 4
        common = dict(seed=i, confidence=0.99, min_iteration_number=0, max_iteration_number=10000)
        corr = dict(common) if lam is None else dict(common, spatial_coherence_weight=lam)
        if k == 0:
            c, _, _, thr = S.problem_h(size, 0.5, seed=seed + i)
            out.append(dict(kind="homography", correspondences=c, threshold=thr, **corr))
        elif k == 1:
            c, _, _, thr = S.problem_f(size, 0.5, seed=seed + i)
            out.append(dict(kind="fundamental", correspondences=c, threshold=thr, **corr))
        elif k == 2:
            fs, fo, _, _, ts, to = S.problem_m2(size // 2, size - size // 2, seed=seed + i)
            out.append(dict(kind="sift", scale_features=fs, orientation_features=fo, scale_residual_thresh=ts,
                            orientation_residual_thresh=to, **common))
        else:
            f, _, thr = S.problem_m1(size, seed=seed + i)
            out.append(dict(kind="scale_only", features=f, scale_residual_thresh=thr, **common))
    return out


def bench_batch(args, rank, world, dist, device, coll_dev):
    """configs[4]: the job's problems LPT-sharded over the ranks, each rank's
    share solved by gcr_solve_batch, one all_gather of the result records."""
    from pygcransac import distributed as D
    from pygcransac import _native as N

    problems = batch_problems(args.problems, lam=args.batch_lambda)
    solve_many = D.batch_solver(device, args.concurrency)
    shares = D.assign_lpt([D.problem_cost(p) for p in problems], world)
    # untimed warm-up: the share's 2 x concurrency costliest problems, so that
    # every solving thread's context exists and its workspace has grown to
    # the largest problem before the timed job (a single warm-up problem
    # left 7 of 8 contexts and their device allocations to the timed region:
    # 290 vs 210 ms per 1024 problems, tools/batch_split.py)
    costs = [D.problem_cost(problems[i]) for i in shares[rank]]
    top = sorted(range(len(costs)), key=lambda j: -costs[j])[:max(2 * args.concurrency, args.warmup // 50)]
    warm = [problems[shares[rank][j]] for j in sorted(top)]
    solve_many(warm)

    def barrier():
        N.check(N.lib.gcr_synchronize(N.context(device)))
        if dist is not None:
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    recs, local = D.solve_sharded(problems, rank=rank, world=world, dist=dist, device=coll_dev,
                                  solve_many=solve_many)
    barrier()
    elapsed = time.perf_counter() - t0
    hyps = float(sum(r["hypotheses"] for r in recs if r is not None))
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    solved = sum(1 for r in recs if r is not None)
    # this rank's per-phase times summed over its problems, per kind (the
    # engine's gcr_stats of each call; wall time overlaps across the
    # concurrent solving threads, so the sums exceed the elapsed time)
    phase_keys = ("ms_setup", "ms_generate", "ms_score", "ms_score_kernel", "ms_replay", "ms_lo", "ms_lo_lists",
                  "ms_lo_fit", "ms_lo_score", "ms_refit_fit", "ms_refit", "ms_total")
    phases = {}
    for i, res in local.items():
        kind = problems[i]["kind"]
        agg = phases.setdefault(kind, dict(problems=0, hypotheses=0, graph_cut_number=0,
                                           **{k: 0.0 for k in phase_keys}))
        st = res["stats"]
        agg["problems"] += 1
        agg["hypotheses"] += int(st["hypotheses"])
        agg["graph_cut_number"] += int(st["graph_cut_number"])
        for k in phase_keys:
            agg[k] += float(st[k])
    if rank == 0:
        print(json.dumps({
            "metric": METRIC,
            "value": hyps / elapsed,
            "unit": "hypotheses/s",
            "n_gpus": world,
            "steps": 1,
            "warmup": len(warm),
            "ms_per_step": elapsed * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (pygcransac/synthetic.py generators, seeded)",
            "config": {"workload": f"configs[4] batch of {len(problems)} independent problems "
                                   "(homography / fundamental / hybrid / scale-only, N ~ U{1000..10000}, "
                                   "50% outliers, confidence 0.99, full estimator calls)",
                       "parallelism": f"LPT problem sharding x{world}, {args.concurrency} host threads per GPU",
                       "problems_per_s": len(problems) / elapsed, "solved": solved,
                       "spatial_coherence_weight_hf": 0.975 if args.batch_lambda is None else args.batch_lambda,
                       "rank0_phase_ms_sums": phases},
            "roofline": None,
            "cpu_baseline": None,
        }))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
