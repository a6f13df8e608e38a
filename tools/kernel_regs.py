#!/usr/bin/env python3
"""VGPR / spill / LDS usage of the built gfx950 kernels (from the code object
inside graph-cut-ransac_amd/csrc/_build/<obj>.o).  usage: kernel_regs.py [substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
OBJ = os.path.join(os.path.dirname(__file__), "..", "graph-cut-ransac_amd", "csrc", "_build", os.environ.get("KOBJ", "kernels.o"))


def main():
    pats = sys.argv[1:]
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", OBJ, os.path.join(d, "x.o")])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", co], text=True)
    recs, cur = [], {}
    for ln in notes.splitlines():
        m = re.match(r"\s+\.(name|vgpr_count|vgpr_spill_count|group_segment_fixed_size|private_segment_fixed_size"
                     r"|sgpr_spill_count):\s+(\S+)", ln)
        if not m:
            continue
        k, v = m.groups()
        if k == "group_segment_fixed_size" and "name" in cur:
            recs.append(cur)
            cur = {}
        cur[k] = v
    recs.append(cur)
    for r in recs:
        n = r.get("name", "")
        mm = re.search(r"(k_\w+?)I(.*?)EEEv", n) or re.search(r"(k_\w+?)E", n)
        short = (mm.group(1) + "<" + re.sub(r"Li|ELb|EL", ",", mm.group(2)).strip(",") + ">") if mm and mm.lastindex == 2 \
            else (mm.group(1) if mm else n[:50])
        if pats and not any(p in short for p in pats):
            continue
        print(f"{short:34s} vgpr {r.get('vgpr_count'):>4} spill {r.get('vgpr_spill_count'):>3} "
              f"lds {r.get('group_segment_fixed_size'):>7} scratch {r.get('private_segment_fixed_size')}")


if __name__ == "__main__":
    main()
