#!/usr/bin/env python3
"""Summarise scripts/pmc_deep.sh output (<dir>/<cfg>_g<i>/run_counter_collection.csv): mean per
launch of the timed render kernel instance, plus derived ratios.
Usage: python scripts/pmc_deep_summary.py <dir> C3 C4"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
for cfg in sys.argv[2:]:
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, f"{cfg}_g*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if "render_kernel<false" not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    print(cfg)
    for k in sorted(m):
        print(f"  {k:24s} {m[k]:.6g}")
    g = m.get
    if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
        print(f"  VALU lane utilisation   {g('SQ_THREAD_CYCLES_VALU') / (64 * g('SQ_ACTIVE_INST_VALU')):.3f}")
    if g("SQ_INSTS_SALU") and g("SQ_INSTS_VALU"):
        print(f"  SALU per VALU           {g('SQ_INSTS_SALU') / g('SQ_INSTS_VALU'):.3f}")
    if g("SQ_WAVE_CYCLES") and g("SQ_WAIT_INST_ANY"):
        print(f"  WAIT_INST_ANY / WAVE_CYCLES {g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
    if g("SQ_INSTS_VALU"):
        print(f"  VALU-issue bound ms     {g('SQ_INSTS_VALU') * 2 / (1024 * 2.4e9) * 1e3:.4f}")
