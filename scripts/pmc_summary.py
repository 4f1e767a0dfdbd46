#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (gpurun_out/<tag>/p*/run_counter_collection.csv) for the
render kernel: per-dispatch means and derived ratios. Usage: python scripts/pmc_summary.py <dir>"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
vals = collections.defaultdict(list)
dur = []
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        # the timed (stats-free) instance; older profiles have a single render_kernel
        if "render_kernel" not in r["Kernel_Name"] or "render_kernel<true" in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
out = dict(counters=m)
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
if g("GRBM_GUI_ACTIVE") and dur:
    out["approx_clock_ghz"] = g("GRBM_GUI_ACTIVE") / 8 / (sum(dur) / len(dur))
if g("FETCH_SIZE") is not None:
    out["fetch_bytes"] = g("FETCH_SIZE") * 1024
if g("WRITE_SIZE") is not None:
    out["write_bytes"] = g("WRITE_SIZE") * 1024
out["mean_dispatch_ns_under_pmc"] = sum(dur) / max(1, len(dur))
print(json.dumps(out, indent=1))
