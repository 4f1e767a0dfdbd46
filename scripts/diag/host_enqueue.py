"""Host enqueue cost of bench.py's frame loop (FrameTiler, two parts, C3) against the GPU time of
the same frames: the part streams are first held by a GPU sleep so that every launch queues up
before any runs; then the frames' GPU time is measured without host starvation. Repeats a few
times to show the host's warm-up.
Usage: python scripts/diag/host_enqueue.py"""
import os
import sys
import time

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
for _ in range(3):
    t.frame()
t.finish()
torch.cuda.synchronize()
for rep in range(6):
    n = 20
    # free-running: host enqueue vs GPU time as the bench times it
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    h0 = time.perf_counter()
    for _ in range(n):
        t.frame()
    h1 = time.perf_counter()
    t.finish()
    e1.record(s)
    torch.cuda.synchronize()
    free_gpu = e0.elapsed_time(e1) / n
    host_free = (h1 - h0) * 1e3 / n
    # queued: hold every part stream with a GPU sleep, enqueue, then time the GPU work only
    for st in t.part_streams:
        st.wait_stream(s)
    with torch.cuda.stream(s):
        torch.cuda._sleep(int(200e6))   # ~0.1 s at ~2 GHz
    hold = s.record_event()
    for st in t.part_streams:
        st.wait_event(hold)
    q0, q1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    q0.record(s)
    h0 = time.perf_counter()
    for _ in range(n):
        t.frame()
    h1 = time.perf_counter()
    t.finish()
    q1.record(s)
    torch.cuda.synchronize()
    print(f"rep {rep}: free-running {free_gpu:.4f} ms/frame GPU, host enqueue {host_free:.4f} ms/frame; "
          f"queued up: host enqueue {(h1 - h0) * 1e3 / n:.4f} ms/frame, GPU {q0.elapsed_time(q1) / n:.4f} "
          f"ms/frame", flush=True)
