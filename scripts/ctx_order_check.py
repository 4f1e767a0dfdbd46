#!/usr/bin/env python3
"""Diagnostic: does a context created after another one (in the same process) render the same
image, at the same speed, as a context in a fresh process? Renders each config of --order in its
own Renderer, one after the other, and reports per-config ms/frame (single stream, back-to-back
launches) and whether the image equals the one saved by a fresh-process run (--save/--check).
Usage: python scripts/ctx_order_check.py --order C3 --save DIR ; python scripts/ctx_order_check.py
       --order C1,C3 --check DIR"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import voxelraytracer_amd as vrt  # noqa: E402
from bench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", default="C1,C3")
    ap.add_argument("--save", default="")
    ap.add_argument("--check", default="")
    ap.add_argument("--frames", type=int, default=200)
    a = ap.parse_args()
    for cfg in a.order.split(","):
        scene, n, w, h, R, T, _ = CONFIGS[cfg]
        with vrt.Renderer(0) as ren:
            ren.upload_volume(vrt.build_scene(scene, n), n)
            cam = vrt.make_camera(w, h)
            p = vrt.default_params(R, T)
            out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
            st = torch.cuda.current_stream()
            for _ in range(50):
                ren.render_rows_async(cam, p, 0, h, 1, out.data_ptr(), stream=st.cuda_stream)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.frames):
                ren.render_rows_async(cam, p, 0, h, 1, out.data_ptr(), stream=st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            img = out.cpu().numpy()
            msg = ""
            if a.save:
                os.makedirs(a.save, exist_ok=True)
                np.save(os.path.join(a.save, f"{cfg}.npy"), img)
            if a.check:
                ref = np.load(os.path.join(a.check, f"{cfg}.npy"))
                msg = f" identical_to_fresh_process={bool(np.array_equal(img, ref))}"
            print(f"{cfg}: {e0.elapsed_time(e1) / a.frames:.4f} ms/frame{msg}", flush=True)


if __name__ == "__main__":
    main()
