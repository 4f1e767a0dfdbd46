"""Diagnostic: how much of a C3 frame the glass pixels cost. Pipelined device-output frames
(vrt_render_frame_device) of the C3 view with the centre voxel as glass (the real scene), stone,
or air; GPU time per frame from events around 300 frames after 300 warm-up."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import voxelraytracer_amd as vrt

def run(vox, n, R=4, T=4, frames=300, warm=300):
    cam = vrt.make_camera(1920, 1080)
    p = vrt.default_params(R, T)
    s = torch.cuda.Stream()
    with vrt.Renderer(0) as r:
        r.upload_volume(vox, n)
        for _ in range(warm):
            r.render_frame_device(cam, p, 1.0, s.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(frames):
            r.render_frame_device(cam, p, 1.0, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / frames

n = 128
base = vrt.build_scene("refraction", n)
c = n // 2
idx = c + c * n + c * n * n
assert base[idx] == 2
for name, v in (("glass (C3)", 2), ("stone", 1), ("air", 0)):
    vox = base.copy()
    vox[idx] = v
    print(f"{name:12s} {run(vox, n):.4f} ms/frame", flush=True)
