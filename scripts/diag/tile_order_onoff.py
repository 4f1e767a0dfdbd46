"""Pipelined device-output frames at C3 with the heavy-first tile order on and off."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import voxelraytracer_amd as vrt

cam = vrt.make_camera(1920, 1080)
p = vrt.default_params(4, 4)
s = torch.cuda.Stream()
for on in (True, False, True, False):
    with vrt.Renderer(0) as r:
        r.set_tile_order(on)
        r.upload_volume(vrt.build_scene("refraction", 128), 128)
        for _ in range(300):
            r.render_frame_device(cam, p, 1.0, s.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(500):
            r.render_frame_device(cam, p, 1.0, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        print("tile order", on, f"{e0.elapsed_time(e1) / 500:.4f} ms/frame", flush=True)
