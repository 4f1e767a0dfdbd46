#!/usr/bin/env python3
"""Certified-walk outcome counts per config from the diagnostic build (make variant NAME=certdiag
DEFS=-DVRT_CERT_DIAG; run with VRT_LIB=build/variants/libvrt_certdiag.so): one stats-free frame.
Usage: VRT_LIB=build/variants/libvrt_certdiag.so python scripts/cert_diag.py [--configs C1,C2,C3,C4]"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import voxelraytracer_amd as vrt  # noqa: E402
from voxelraytracer_amd import abi  # noqa: E402
from bench import CONFIGS  # noqa: E402

NAMES = ["exact_start", "primary_unsure", "miss", "glass_hit", "hit_ambient", "back_face",
         "shadow_start_unsure", "air_cell", "shadow_unsure", "shadow_certified",
         "primary_iters", "glass_tree_certified", "primary_wave_max_iters"]
# certified bounce trees (slots 16-31; the shade counters 4-9 above also count the trees' hits)
TREE = {16: "tree_attempted", 17: "tree_certified", 18: "tree_two_pending", 19: "tree_reflection_start",
        20: "tree_refraction_start", 21: "tree_march_unsure", 22: "tree_shade_unsure", 23: "tree_rays_certified",
        24: "march_fastpath_or_e0", 25: "march_walk_unsure", 26: "ivr_point_not_robust", 27: "ivr_noise",
        28: "ivr_start", 29: "march_seg_limit", 30: "ivr_count", 31: "tree_start_cell_outside"}
ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="C1,C2,C3,C4")
args = ap.parse_args()
lib = abi.load_library()
lib.vrt_debug_cert_diag.argtypes = [C.c_void_p]
dev = torch.device("cuda", 0)
for cfg in args.configs.split(","):
    scene, n, w, h, R, T, _ = CONFIGS[cfg]
    vox = torch.from_numpy(vrt.build_scene(scene, n)).to(dev)
    out = torch.empty((h, w, 4), dtype=torch.float32, device=dev)
    cnt = np.zeros(32, np.uint64)
    with vrt.Renderer(0) as ren:
        ren.upload_volume_device(vox.data_ptr(), n, 0)
        torch.cuda.synchronize()
        assert lib.vrt_debug_cert_diag(cnt.ctypes.data) == 0   # reset
        ren.render_rows_async(vrt.make_camera(w, h), vrt.default_params(R, T), 0, h, 1,
                              out.data_ptr(), 0, 0, 0)
        torch.cuda.synchronize()
        assert lib.vrt_debug_cert_diag(cnt.ctypes.data) == 0
    px = w * h
    d = {k: round(float(cnt[i]) / px, 5) for i, k in enumerate(NAMES)}
    d["primary_wave_max_iters"] = round(float(cnt[12]) / (px / 64), 3)
    certified = (cnt[2] + cnt[4] + cnt[9]) / px
    tree = {v: int(cnt[k]) for k, v in TREE.items()}
    if cnt[16]:
        tree["tree_certified_frac"] = round(float(cnt[17]) / float(cnt[16]), 5)
    print(cfg, json.dumps(dict(pixels=px, certified=round(float(certified), 5), **d, tree=tree)), flush=True)
