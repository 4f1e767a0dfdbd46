"""GPU time of each of the first 30 frames of a fresh process (C3, FrameTiler, two parts), each
frame joined before the next (no overlap): which frames carry one-off costs."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import voxelraytracer_amd as vrt  # noqa: E402
from voxelraytracer_amd.tiles import FrameTiler, row_pitch  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_stream(torch.cuda.Stream(device=dev))
s = torch.cuda.current_stream(dev)
ren = vrt.Renderer(0)
ren.upload_volume(vrt.build_scene("refraction", 128), 128)
cam = vrt.make_camera(1920, 1080)
p = vrt.default_params(4, 4)


def band(row0, rows, step, out, prev):
    sp = torch.cuda.current_stream(dev).cuda_stream
    ren.render_temporal_rows_async(cam, p, 1.0, row0, rows, step, prev.data_ptr(), out.data_ptr(),
                                   0, 0, 0, sp, pitch=row_pitch(out))


t = FrameTiler(1920, 1080, band, dev, dtype=torch.uint8, parts=2)
torch.cuda.synchronize()
evs = []
for i in range(30):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    t.frame()
    t.finish()
    e1.record(s)
    evs.append((e0, e1))
torch.cuda.synchronize()
print("ms per frame:", " ".join(f"{a.elapsed_time(b):.3f}" for a, b in evs), flush=True)
