#!/usr/bin/env python3
"""Copy one scripts/gpu_check.sh run (gpurun_out/<tag>/) into profiles/: the rocprofv3 kernel
stats and bench line, the PMC passes with their summary, and profiles/pmc_<cfg>_<output>.json
(hbm_bytes_per_launch of the timed render kernel, read by bench.py as roofline.traffic).
FETCH_SIZE is doubled per MI355X_MICROARCH.md's gfx950 correction; WRITE_SIZE is taken as is.
Usage: python scripts/save_profiles.py <tag> [--config C3] [--output rgba8]"""
import argparse
import re
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("tag")
ap.add_argument("--config", default="C3")
ap.add_argument("--output", default="rgba8")
a = ap.parse_args()
src = os.path.join(ROOT, "gpurun_out", a.tag)
dst = os.path.join(ROOT, "profiles", a.tag if re.match(r"r\d\d_", a.tag) else f"r02_{a.tag}")
os.makedirs(dst, exist_ok=True)
for name in ("bench.log", "pytest_gpu.log", "smoke.log"):
    p = os.path.join(src, name)
    if os.path.exists(p):
        with open(p) as f, open(os.path.join(dst, name), "w") as g:
            g.writelines(l for l in f if "amdgpu.ids" not in l)
pt = os.path.join(src, "prof_trace.log")   # the bench line printed under the kernel trace
if os.path.exists(pt):
    lines = [l for l in open(pt) if l.startswith("{")]
    if lines:
        with open(os.path.join(dst, "bench_under_rocprof.json"), "w") as g:
            g.write(lines[-1])
ks = os.path.join(src, "trace", "run_kernel_stats.csv")
if os.path.exists(ks):
    shutil.copy(ks, os.path.join(dst, f"{a.config}_kernel_stats.csv"))
passes = [d for d in ("pmc_fetch", "pmc_write", "pmc_sq")
          if os.path.exists(os.path.join(src, d, "run_counter_collection.csv"))]
if passes:
    tmp = os.path.join(dst, "pmc")
    for d in passes:
        os.makedirs(os.path.join(tmp, "p_" + d[4:]), exist_ok=True)
        shutil.copy(os.path.join(src, d, "run_counter_collection.csv"),
                    os.path.join(tmp, "p_" + d[4:], "run_counter_collection.csv"))
    summ = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), tmp],
                          check=True, capture_output=True, text=True).stdout
    with open(os.path.join(tmp, "summary.json"), "w") as f:
        f.write(summ)
    s = json.loads(summ)
    if "fetch_bytes" in s and "write_bytes" in s:
        out = {"config": a.config, "output": a.output,
               "kernel": "one frame's launch, its kernels summed: " + " + ".join(
                   sorted(k for k in s.get("per_kernel", {}) if "render" in k or "exact" in k)),
               "source": f"profiles/{os.path.basename(dst)}/pmc (rocprofv3 --pmc FETCH_SIZE and --pmc "
                         "WRITE_SIZE in separate passes over bench.py --steps 5 --warmup 1 "
                         "--device-warmup-ms 0: one launch = one frame)",
               "fetch_size_bytes_raw": s["fetch_bytes"], "write_size_bytes": s["write_bytes"],
               "correction": "gfx950: FETCH_SIZE reports half the bytes of 128-B requests "
                             "(MI355X_MICROARCH.md HBM section) -> doubled; WRITE_SIZE as is",
               "hbm_bytes_per_launch": int(2 * s["fetch_bytes"] + s["write_bytes"]),
               "parts": 1}
        shp = os.path.join(src, "lib.sha256")
        if os.path.exists(shp):   # the build the passes measured; bench.py refuses other builds
            out["lib_sha256"] = open(shp).read().strip()
        if s.get("counters", {}).get("SQ_INSTS_VALU"):
            out["valu_insts_per_launch"] = int(s["counters"]["SQ_INSTS_VALU"])
        with open(os.path.join(ROOT, "profiles", f"pmc_{a.config}_{a.output}.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out))
print("saved", dst)
