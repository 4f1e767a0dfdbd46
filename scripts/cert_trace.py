#!/usr/bin/env python3
"""Diagnostic: the certified walks of one pixel (a VRT_CERT_TRACE build, make variant NAME=trace
DEFS="-DVRT_CERT_TRACE -DVRT_TRACE_PX=x -DVRT_TRACE_PY=y", loaded by VRT_LIB), in lane with the
given certified mode. Records: 100/101 walk start (shadow flag, cell, P, U / D, e0, ed), 102 an
empty-space box (G, s1, uj, gam), 103/104 a crossing (next cell, s1, axis, near-edge flags, byte /
cell, sig, gam of the axis). Usage: python scripts/cert_trace.py scene n w h px py pz rx ry R T cert [trees]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraytracer_amd as vrt  # noqa: E402


def main():
    a = sys.argv[1:]
    scene, n, w, h = a[0], int(a[1]), int(a[2]), int(a[3])
    pos = tuple(map(float, a[4:7]))
    rot = (float(a[7]), float(a[8]), 0.0)
    R, T, cert = int(a[9]), int(a[10]), int(a[11])
    trees = int(a[12]) if len(a) > 12 else 0
    lib = vrt.lib()
    lib.vrt_debug_cert_trace.argtypes = [C.c_void_p, C.c_void_p]
    out = np.zeros((1024, 8), np.float32)
    cnt = C.c_uint32()
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene(scene, n), n)
        r.set_certified(cert)
        r.set_cert_trees(trees)
        r.set_exact_pass(0)
        cam = vrt.make_camera(w, h, pos=pos, rot=rot)
        p = vrt.default_params(R, T, time=1.0)
        buf = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda")
        lib.vrt_debug_cert_trace(out.ctypes.data, C.byref(cnt))
        r.render_temporal_rows_async(cam, p, 1.0, 0, h, 1, buf.data_ptr(), buf.data_ptr(),
                                     stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        lib.vrt_debug_cert_trace(out.ctypes.data, C.byref(cnt))
    np.set_printoptions(precision=9, suppress=True, linewidth=220)
    for i in range(min(cnt.value, 1024)):
        print(" ".join(f"{x:.9g}" for x in out[i]))


if __name__ == "__main__":
    main()
