#!/usr/bin/env python3
"""Diagnostic: one frame through every certified mode (certified trees with the deferred exact pass
or in lane, no trees, exact primaries with certified shadow / secondary rays, exact walks only)
against the exact STATS instance; prints the pixels that differ (r06_s19-s21 located the
cert_continuation start-layer case with it). Usage:
python scripts/cert_modes_diag.py [scene n w h px py pz rx ry R T]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraytracer_amd as vrt  # noqa: E402


def frame(r, cam, p, counters=False):
    h, w = cam.height, cam.width
    buf = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(len(vrt.COUNTER_NAMES), dtype=torch.int64, device="cuda")
    r.render_temporal_rows_async(cam, p, 1.0, 0, h, 1, buf.data_ptr(), buf.data_ptr(),
                                 d_counters=cnt.data_ptr() if counters else 0,
                                 stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return buf.cpu().numpy()


def main():
    a = sys.argv[1:]
    scene, n, w, h = (a[0], int(a[1]), int(a[2]), int(a[3])) if a else ("glass_cube", 64, 320, 180)
    pos = tuple(map(float, a[4:7])) if len(a) >= 7 else (1.0, 2.0, -3.0)
    rot = (float(a[7]), float(a[8]), 0.0) if len(a) >= 9 else (0.0, 0.0, 0.0)
    R, T = (int(a[9]), int(a[10])) if len(a) >= 11 else (4, 4)
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene(scene, n), n)
        r.set_certified(1)
        cam = vrt.make_camera(w, h, pos=pos, rot=rot)
        p = vrt.default_params(R, T, time=1.0)
        ref = frame(r, cam, p, counters=True)
        for name, trees, ep, cert in (("trees, deferred", 2, 2, 1), ("trees in lane", 2, 0, 1),
                                      ("no trees, deferred", 0, 2, 1), ("no trees, in lane", 0, 0, 1),
                                      ("exact primary, certified shadow/secondary", 0, 0, 0),
                                      ("exact walks only", 0, 0, -1)):
            r.set_certified(cert)
            r.set_cert_trees(trees)
            r.set_exact_pass(ep)
            got = frame(r, cam, p)
            bad = np.argwhere(np.any(got != ref, axis=-1))
            print(f"{name}: {len(bad)} pixels differ", flush=True)
            for y, x in bad[:8]:
                print(f"   ({x}, {y}) got {got[y, x].tolist()} ref {ref[y, x].tolist()}")


if __name__ == "__main__":
    main()
