#!/usr/bin/env python3
"""Counters of one frame per config from a diagnostic build (VRT_LIB=...): prints all counters.
With the VRT_DIAG_SAMPLED build the TIE3 slot holds the number of sampled fast-path steps.
Usage: VRT_LIB=build/variants/libvrt_diag.so python scripts/diag_counts.py [--configs C1,C2,C3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import voxelraytracer_amd as vrt  # noqa: E402
from bench import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="C1,C2,C3,C4")
args = ap.parse_args()
dev = torch.device("cuda", 0)
for cfg in args.configs.split(","):
    scene, n, w, h, R, T, _ = CONFIGS[cfg]
    vox = torch.from_numpy(vrt.build_scene(scene, n)).to(dev)
    out = torch.empty((h, w, 4), dtype=torch.float32, device=dev)
    cnt = torch.zeros(len(vrt.COUNTER_NAMES), dtype=torch.int64, device=dev)
    with vrt.Renderer(0) as ren:
        ren.upload_volume_device(vox.data_ptr(), n, 0)
        ren.render_rows_async(vrt.make_camera(w, h), vrt.default_params(R, T), 0, h, 1,
                              out.data_ptr(), 0, cnt.data_ptr(), 0)
        torch.cuda.synchronize()
    print(cfg, json.dumps(vrt.counters_dict(cnt.cpu().tolist())))
