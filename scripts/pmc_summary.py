#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (gpurun_out/<tag>/p*/run_counter_collection.csv) for the timed
frame: per-dispatch means of each of its kernels, their per-frame sum and derived ratios.
Usage: python scripts/pmc_summary.py <dir>"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
# the timed launch: the stats-free render_kernel (older profiles: the only render_kernel) and, since
# r03, the deferred exact pass that follows it on the same stream (one frame = one of each)
TIMED = ("render_kernel<false", "exact_pass_kernel")
per = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> counter -> values
durs = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        key = next((t for t in TIMED if t in name), None)
        if key is None:
            continue
        per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        durs[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
kern = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
# per frame: the sum of the kernels' per-dispatch means
m = collections.defaultdict(float)
for k, cs in kern.items():
    for c, v in cs.items():
        m[c] += v
m = dict(m)
out = dict(counters=m, per_kernel=kern)
g = lambda k: m.get(k)
if g("SQ_WAVES"):
    w = g("SQ_WAVES")
    out["valu_per_wave"] = g("SQ_INSTS_VALU") / w if g("SQ_INSTS_VALU") else None
    out["salu_per_wave"] = g("SQ_INSTS_SALU") / w if g("SQ_INSTS_SALU") else None
if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
    out["valu_lane_util"] = g("SQ_THREAD_CYCLES_VALU") / (64 * g("SQ_ACTIVE_INST_VALU"))
if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
    out["l2_hit_rate"] = g("TCC_HIT_sum") / max(1.0, g("TCC_HIT_sum") + g("TCC_MISS_sum"))
if g("SQ_WAVE_CYCLES"):
    for k in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
        if g(k):
            out[k + "_frac_of_wave_cycles"] = g(k) / g("SQ_WAVE_CYCLES")
if g("FETCH_SIZE") is not None:
    out["fetch_bytes"] = g("FETCH_SIZE") * 1024
if g("WRITE_SIZE") is not None:
    out["write_bytes"] = g("WRITE_SIZE") * 1024
out["mean_dispatch_ns_under_pmc"] = {k: sum(v) / max(1, len(v)) for k, v in durs.items()}
print(json.dumps(out, indent=1))
