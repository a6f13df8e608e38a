#!/usr/bin/env python3
"""Loops of one kernel in a hipcc -save-temps gfx950 .s file: for each backward
branch, its body's instruction counts (VALU / SALU / memory) and, with --hist,
the VALU opcode histogram of the biggest loops.
usage: isa_loops.py KERNELS.s NAME_REGEX [--top 6] [--hist 2]"""
import argparse
import collections
import re

ap = argparse.ArgumentParser()
ap.add_argument("s")
ap.add_argument("name")
ap.add_argument("--top", type=int, default=6)
ap.add_argument("--hist", type=int, default=0)
a = ap.parse_args()
src = open(a.s).read()
m = [x for x in re.finditer(r"^(_Z\S*" + a.name + r"\S*):", src, re.M)]
name = m[0].group(1)
start = m[0].end()
body = src[start:src.index(".Lfunc_end", start)].split("\n")
labels = {}
for i, l in enumerate(body):
    mm = re.match(r"^(\.LBB\w+):", l)
    if mm:
        labels[mm.group(1)] = i
loops = []
for i, l in enumerate(body):
    mm = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
        loops.append((labels[mm.group(1)], i, mm.group(1)))


def hist(lo, hi):
    c = collections.Counter()
    for l in body[lo:hi]:
        t = l.strip().split()
        if t and re.match(r"^(v_|s_|global_|ds_|buffer_|flat_)", t[0]):
            c[t[0]] += 1
    return c


print(name)
big = sorted(loops, key=lambda x: x[1] - x[0], reverse=True)
for lo, hi, t in big[:a.top]:
    h = hist(lo, hi)
    print(f"  {t:14s} lines {lo:6d}-{hi:6d} insts {sum(h.values()):5d} valu "
          f"{sum(v for k, v in h.items() if k.startswith('v_')):5d} salu "
          f"{sum(v for k, v in h.items() if k.startswith('s_')):5d} mem "
          f"{sum(v for k, v in h.items() if not k.startswith(('v_', 's_'))):4d}")
for lo, hi, t in big[:a.hist]:
    h = hist(lo, hi)
    print(f"  {t}:")
    for k, v in h.most_common(60):
        print(f"    {k:28s} {v}")
