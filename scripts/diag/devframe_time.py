"""GPU time per frame of pipelined device-output frames (vrt_render_frame_device) at C3, through
the Python binding of the library in VRT_LIB (A/B of context variants)."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import voxelraytracer_amd as vrt

cam = vrt.make_camera(1920, 1080)
p = vrt.default_params(4, 4)
s = torch.cuda.Stream()
with vrt.Renderer(0) as r:
    r.upload_volume(vrt.build_scene("refraction", 128), 128)
    for _ in range(300):
        r.render_frame_device(cam, p, 1.0, s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(500):
        r.render_frame_device(cam, p, 1.0, s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    print(os.path.basename(os.environ.get("VRT_LIB", "base")), f"{e0.elapsed_time(e1) / 500:.4f} ms/frame")
