#!/usr/bin/env python3
"""Per-phase instruction budget of the certified pass from PMC passes of the phase-diagnostic
builds (make variant NAME=phK DEFS=-DVRT_DIAG_PHASE=K; gpu_session.sh steps `sq` and `sca` over
base + build/variants/*.so). Phase K stops the certified pass after: 0 nothing (ray setup
skipped), 1 the primary ray, 2 the primary certified walk, 3 the shading without the shadow walk;
the product library (base) is the whole frame. Differences of consecutive builds are each phase's
cost; counters per frame are the sum of the frame's kernels' per-dispatch means.
Usage: python scripts/phase_budget.py gpurun_out/<tag> [CFG]"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
cfg = sys.argv[2] if len(sys.argv) > 2 else "C3"
TIMED = ("render_kernel<false", "exact_pass_kernel")
PHASES = [("libvrt_ph0", "0 launch + epilogue (no ray setup)"), ("libvrt_ph1", "1 primary ray setup"),
          ("libvrt_ph2", "2 primary certified walk"), ("libvrt_ph3", "3 shading, sky, deferral (no shadow walk)"),
          ("base", "4 shadow walks + deferred exact pass (the product)")]


def per_frame(path):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(path, "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            key = next((t for t in TIMED if t in r["Kernel_Name"]), None)
            if key:
                per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = collections.defaultdict(float)
    for k, cs in per.items():
        for c, v in cs.items():
            out[c] += sum(v) / len(v)
    return dict(out)


rows = []
for lib, what in PHASES:
    m = {}
    for grp in ("sq", "sca"):
        m.update(per_frame(os.path.join(d, f"{grp}_{lib}_{cfg}")))
    rows.append((lib, what, m))
keys = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS",
        "SQ_INSTS_BRANCH", "SQ_ACTIVE_INST_SCA", "SQ_INST_CYCLES_SALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES",
        "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"]
res = {"config": cfg, "phases": []}
prev = None
for lib, what, m in rows:
    e = {"build": lib, "phase": what, "per_frame": {k: m.get(k) for k in keys if k in m}}
    if prev is not None:
        e["delta"] = {k: m[k] - prev[k] for k in keys if k in m and k in prev}
    res["phases"].append(e)
    prev = m
base = rows[-1][2]
if base.get("SQ_INSTS_VALU"):
    cus, simds = 256, 1024
    res["issue_floors_us"] = {
        "valu": base["SQ_INSTS_VALU"] * 2 / (simds * 2.4e3),   # 2 cycles per wave64 VALU on a SIMD32
        "salu_one_per_cu_cycle": base.get("SQ_INSTS_SALU", 0) / (cus * 2.4e3),
        "note": "VALU: 2 cycles per wave64 instruction per SIMD (MI355X_MICROARCH.md); SALU: one "
                "scalar unit per CU at one instruction per cycle",
    }
print(json.dumps(res, indent=1))
