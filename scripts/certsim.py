#!/usr/bin/env python3
"""Driver of scripts/certsim.c (analysis only): certified walks against the exact walks of the
oracle for the primary and shadow rays of a BASELINE config.
Usage: python scripts/certsim.py [--config C3] [--gscale 1] [--margin 0.015625] [--scale 1]"""
import argparse
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import voxelraytracer_amd as vrt  # noqa: E402
from bench import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--gscale", type=float, default=1.0)
ap.add_argument("--margin", type=float, default=1.0 / 64)
ap.add_argument("--scale", type=int, default=1, help="divide the resolution")
ap.add_argument("--cap", type=int, default=64)
a = ap.parse_args()
so = os.path.join(ROOT, "build", "certsim.so")
subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-shared",
                       "-fPIC", "-o", so, os.path.join(ROOT, "scripts", "certsim.c"), "-lm"])
L = C.CDLL(so)
L.cs_build.argtypes = [C.c_void_p, C.c_int, C.c_int]
L.cs_run.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_float, C.c_double, C.c_float,
                     C.c_void_p]
scene, n, w, h, R, T, desc = CONFIGS[a.config]
w //= a.scale
h //= a.scale
vox = vrt.build_scene(scene, n)
cam = vrt.make_camera(w, h)
p = vrt.default_params(R, T)
sun = np.array(p.sun_dir[:], np.float32)
L.cs_build(vox.ctypes.data, n, a.cap)
inv = np.array(cam.inv_pv[:], np.float32)
o = np.zeros(32, np.float64)
L.cs_run(inv.ctypes.data, w, h, sun.ctypes.data, C.c_float(p.max_ray_length), a.gscale,
         C.c_float(a.margin), o.ctypes.data)
px = o[0]
print(f"{a.config} {w}x{h} gscale {a.gscale} margin {a.margin}")
print(f"  primary: exact steps/ray {o[1]/px:.1f}; certified iters/ray {o[2]/px:.2f} "
      f"(jumps {o[3]/px:.2f}); uncertain {o[4]/px:.4%} (why {o[20:24].astype(int).tolist()}); "
      f"miss {o[5]:.0f} hit {o[7]:.0f} MISMATCH {o[6]:.0f}")
sh = max(o[8], 1)
print(f"  shadow:  rays {o[8]:.0f}, exact steps/ray {o[9]/sh:.1f}; irrelevant {o[10]/sh:.2%}; "
      f"primary-uncertain {o[11]/sh:.2%}; back-face {o[12]/sh:.2%}; start-uncertain {o[13]/sh:.2%}; "
      f"certified iters/ray {o[14]/max(o[17]+o[16],1):.2f} (jumps {o[15]/max(o[17]+o[16],1):.2f}); "
      f"uncertain {o[16]/sh:.3%} (why {o[24:28].astype(int).tolist()}); certified {o[17]/sh:.2%} MISMATCH {o[18]:.0f}")
print(f"  pixels needing the exact path: {o[19]/px:.3%}; 8x8 waves with one: {o[30]:.2%} "
      f"(primary only {o[31]:.2%})")
