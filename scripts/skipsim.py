#!/usr/bin/env python3
"""Driver of scripts/skipsim.c (analysis only): sampled-step counts of the centred vs octant
empty-space schemes for the primary + shadow walks of a BASELINE config.
Usage: python scripts/skipsim.py [--config C3] [--stride 1] [--capc 64] [--capo 255]"""
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
ap.add_argument("--stride", type=int, default=1, help="simulate every k-th 8x8 tile")
ap.add_argument("--capc", type=int, default=64)
ap.add_argument("--capo", type=int, default=255)
a = ap.parse_args()
so = os.path.join(ROOT, "build", "skipsim.so")
subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fopenmp", "-shared", "-fPIC", "-o", so,
                       os.path.join(ROOT, "scripts", "skipsim.c")])
L = C.CDLL(so)
L.sim_build.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
L.sim_run.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_float, C.c_void_p]
scene, n, w, h, R, T, desc = CONFIGS[a.config]
vox = vrt.build_scene(scene, n)
cam = vrt.make_camera(w, h)
p = vrt.default_params(R, T)
sun = np.array(p.sun_dir[:], np.float32)
sun_n = (sun * (np.float32(1) / np.sqrt(np.float32(sun[0] * sun[0] + sun[1] * sun[1] + sun[2] * sun[2])))).astype(np.float32)
L.sim_build(vox.ctypes.data, n, a.capc, a.capo)
inv = np.array(cam.inv_pv[:], np.float32)
out = np.zeros(4 + 4 * 4, np.float64)
L.sim_run(inv.ctypes.data, w, h, a.stride, sun_n.ctypes.data, C.c_float(p.max_ray_length), out.ctypes.data)
lp, ls, wp, ws = out[:4]
print(f"{a.config} {desc}: lane steps prim {lp:.3e} shadow {ls:.3e}; wave steps prim {wp:.3e} shadow {ws:.3e}")
for sc, name in enumerate(["centred D", "octant F", "guarded F'", "G ? F : F'"]):
    o = out[4 + 4 * sc: 8 + 4 * sc]
    valu = (wp + ws) * 24 + (o[2] + o[3]) * 50
    print(f"  {name:10s}: lane samples prim {o[0]:.3e} ({o[0]/lp:.1%}) shadow {o[1]:.3e} ({o[1]/max(ls,1):.1%}); "
          f"wave samples prim {o[2]:.3e} ({o[2]/wp:.1%}) shadow {o[3]:.3e} ({o[3]/max(ws,1):.1%}); est VALU {valu:.3e}")
