#!/usr/bin/env python3
"""Static VALU opcode mix of the built gfx950 kernels, for bench.py's VALU-issue
roofline (roofline.valu_issue): the "other" bucket (VALU instructions outside
the SQ_INSTS_VALU_* class counters) is split by the kernel's opcode histogram
and each opcode priced from tools/micro/valu_issue.hip.

The code object comes from graph-cut-ransac_amd/csrc/_build/kernels.o (the
object libgcr.so is linked from).  rocprofv3 gives no per-block execution
counts, so each kernel is cut into regions -- every loop (a backward branch)
and the straight code outside them, each instruction in its innermost loop --
with per region its static VALU count, its counts per SQ_INSTS_VALU_* class and
its other-bucket opcode histogram.  bench.py fits each region's execution
count (non-negative least squares) to the PMC class counts of the same build
and so splits the measured other bucket by opcode.  Written to
profiles/valu_mix.json keyed by kernel name, with the library's kernel build id.
usage: valu_mix.py [kernel-substring ...] [--out profiles/valu_mix.json]"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(REPO, "graph-cut-ransac_amd", "csrc", "_build", "kernels.o")

# opcode -> PMC class counted by SQ_INSTS_VALU_<class> (None: the "other" bucket)
def pmc_class(op):
    o = op.split("_e32")[0].split("_e64")[0].split("_sdwa")[0].split("_dpp")[0]
    if re.match(r"v_(add|sub|subrev)_f64$", o): return "ADD_F64"
    if re.match(r"v_mul_f64$", o): return "MUL_F64"
    if re.match(r"v_(fma|fmac)_f64$", o): return "FMA_F64"
    if re.match(r"v_(rcp|rsq|sqrt)_f64$", o): return "TRANS_F64"
    if re.match(r"v_(add|sub|subrev|pk_add)_f32$", o): return "ADD_F32"
    if re.match(r"v_(mul|pk_mul)_f32$", o): return "MUL_F32"
    if re.match(r"v_(fma|fmac|mac|mad|pk_fma)_f32$", o): return "FMA_F32"
    if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32$", o): return "TRANS_F32"
    if re.match(r"v_cvt_", o): return "CVT"
    if re.match(r"v_(lshl_add|lshlrev|lshrrev|ashrrev|add|sub|mad)_u64|v_mad_u64_u32|v_mad_i64_i32|v_lshl_add_u64", o):
        return "INT64"
    if re.match(r"v_(add|sub|subrev|add3|mul_lo|mul_hi|mad|lshl_add|add_lshl|lshl_or|and_or|or3|xad|mul_u32|mul_i32)"
                r"_(u32|i32|co_u32|co_ci_u32|u16|i16|b32)$", o) or re.match(r"v_(addc|subb|subbrev)_co_u32$", o):
        return "INT32"
    return None


def disasm():
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", OBJ, os.path.join(d, "x.o")])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        return subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], text=True)


def short_name(sym):
    """k_score_fm<2, 16, true> (bench.py's kernel names) from the mangled symbol"""
    mm = re.search(r"(k_\w+?)I(.*?)EEEv", sym)
    if mm:
        args = re.findall(r"Li(\d+)E|Lb([01])E|Lj(\d+)E", mm.group(2) + "E")
        vals = [x[0] or x[2] or ("true" if x[1] == "1" else "false") for x in args]
        return f"{mm.group(1)}<{', '.join(vals)}>"
    mm = re.search(r"(k_\w+?)E", sym)
    return mm.group(1) if mm else sym[:60]


def parse_kernels(text, want):
    """{short name: [(addr, opcode, backward-branch target or None)]}"""
    out, cur = {}, None
    for ln in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", ln)
        if m:
            cur = short_name(m.group(1))
            if want and not any(k in cur for k in want):
                cur = None
            else:
                out[cur] = []
            continue
        if cur is None:
            continue
        t = ln.strip().split()
        mm = re.search(r"// ([0-9A-Fa-f]+):", ln)
        if not t or not mm:
            continue
        addr = int(mm.group(1), 16)
        tgt = None
        mb = re.search(r"<\S+\+0x([0-9a-f]+)>", ln)
        if t[0].startswith(("s_cbranch", "s_branch")) and mb:
            tgt = mb.group(1)
        out[cur].append([addr, t[0], tgt])
    # branch targets are symbol-relative offsets: rebase on the symbol start
    for k, ins in out.items():
        if not ins:
            continue
        base = ins[0][0]
        for e in ins:
            if e[2] is not None:
                e[2] = base + int(e[2], 16)
    return out


def regions(ins):
    """Each instruction's innermost loop (a backward branch's [target, branch]);
    region 0 is the code outside every loop.  Per region: VALU total, the
    PMC-class counts and the other bucket's opcode histogram."""
    loops = sorted({(e[2], e[0]) for e in ins if e[2] is not None and e[2] <= e[0]}, key=lambda l: l[1] - l[0])
    regs = [{"lo": None, "hi": None, "valu": 0, "classes": collections.Counter(), "other": collections.Counter()}]
    regs += [{"lo": lo, "hi": hi, "valu": 0, "classes": collections.Counter(), "other": collections.Counter()}
             for lo, hi in loops]
    for addr, op, _ in ins:
        if not op.startswith("v_"):
            continue
        r = 0
        for i, (lo, hi) in enumerate(loops):      # smallest enclosing loop first
            if lo <= addr <= hi:
                r = i + 1
                break
        g = regs[r]
        g["valu"] += 1
        cl = pmc_class(op)
        if cl:
            g["classes"][cl] += 1
        else:
            g["other"][op] += 1
    return [dict(g, classes=dict(g["classes"]), other=dict(g["other"])) for g in regs if g["valu"] > 0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels", nargs="*")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "valu_mix.json"))
    a = ap.parse_args()
    sys.path.insert(0, os.path.join(REPO, "graph-cut-ransac_amd"))
    from pygcransac import _native as N
    build = N.lib.gcr_kernel_build_id().decode()
    ks = parse_kernels(disasm(), a.kernels)
    res = {}
    for k, ins in ks.items():
        regs = regions(ins)
        res[k] = {"kernel_build_id": build, "regions": regs,
                  "valu_static": sum(g["valu"] for g in regs)}
    prev = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            prev = json.load(f)
    prev.update(res)
    with open(a.out, "w") as f:
        json.dump(prev, f, indent=1, sort_keys=True)
    for k, v in res.items():
        print(f"{k:40s} valu {v['valu_static']:6d} regions {len(v['regions'])}")


if __name__ == "__main__":
    main()
