"""Do the two part streams' launches run in lockstep, and does staggering them help? C3 frames
through bench.py's FrameTiler (two parts), steady state, after an initial GPU sleep of S cycles on
part stream 1 only (S = 0: no stagger).
Usage: python scripts/diag/stagger.py S [S ...]"""
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


for arg in sys.argv[1:] or ["0"]:
    cycles = int(arg)
    t = FrameTiler(1920, 1080, band, dev, dtype=torch.uint8, parts=2)
    for _ in range(300):
        t.frame()
    t.finish()
    torch.cuda.synchronize()
    for st in t.part_streams:
        st.wait_stream(s)
    if cycles:
        with torch.cuda.stream(t.part_streams[1]):
            torch.cuda._sleep(cycles)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(50):   # let the stagger settle in
        t.frame()
    e0.record(t.part_streams[0])   # part stream 0 has finished the settle frames
    n = 500
    for _ in range(n):
        t.frame()
    t.finish()
    e1.record(s)
    torch.cuda.synchronize()
    print(f"stagger {cycles} cycles: {e0.elapsed_time(e1) / n:.4f} ms/frame", flush=True)
