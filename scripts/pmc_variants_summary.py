#!/usr/bin/env python3
"""Mean per launch of every counter of the stats-free colour-only render kernel (and the queue
kernel), per variant directory written by scripts/pmc_variants.sh.
Usage: python scripts/pmc_variants_summary.py DIR"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
runs = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "*_g*", "run_counter_collection.csv"))):
    var = os.path.basename(os.path.dirname(f)).rsplit("_g", 1)[0]
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"]
        if "render_kernel<false, false" in kn:
            key = "main"
            runs[var][(key, r["Counter_Name"])].append(float(r["Counter_Value"]))
for var, m in runs.items():
    print(var)
    for (k, c), v in sorted(m.items()):
        print(f"  {k:5s} {c:24s} {sum(v) / len(v):.6g}")
