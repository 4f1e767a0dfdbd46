#!/usr/bin/env python3
"""List the scratch (spill / private array) stores of one render_kernel instance in the gfx950
assembly (make asm -> build/asm/vrt_render.s), with the basic block each sits in.
Usage: python scripts/scratch_ops.py [instance-substring, default ILb0ELb0ELi2E] [--loads]"""
import re
import sys

inst = next((a for a in sys.argv[1:] if not a.startswith("--")), "ILb0ELb0ELi2E")
loads = "--loads" in sys.argv
s = open("build/asm/vrt_render.s").read().split("\n")
i = [k for k, l in enumerate(s) if l.startswith("_ZN3vrt13render_kernel" + inst)][0]
j = i
while not s[j].startswith(".Lfunc_end"):
    j += 1
lab = None
n = 0
for k in range(i, j):
    l = s[k]
    if re.match(r"^\.LBB\d+_\d+:", l) or l.startswith("; %bb."):
        lab = l.strip()
    if "scratch_store" in l or (loads and "scratch_load" in l):
        n += 1
        print(f"{k - i:6d} {lab:14s} {l.strip()[:70]}")
print(f"{n} scratch ops in {j - i} lines")
