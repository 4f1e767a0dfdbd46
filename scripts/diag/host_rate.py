"""Host enqueue cost per frame against the GPU time per frame, for C3's band of a k-GPU split
(k = 1, 8) with four lanes: is a small band's frame rate bound by the host?
  tiler : bench.py's FrameTiler (Python, torch stream contexts, ctypes per launch)
  raw   : the same launches from a bare Python loop (ctypes only)
  dev   : vrt_render_frame_device of a one-device context (the C++ lanes), whole frame only
Prints host ms/frame (wall time of the enqueue loop, no sync inside) and GPU ms/frame (events).
Usage: python scripts/diag/host_rate.py"""
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import voxelraytracer_amd as vrt  # noqa: E402
from voxelraytracer_amd.tiles import FrameTiler, row_pitch  # noqa: E402

W, H = 1920, 1080
dev = torch.device("cuda", 0)
torch.cuda.set_stream(torch.cuda.Stream(device=dev))
main = torch.cuda.current_stream(dev)
ren = vrt.Renderer(0)
ren.upload_volume(vrt.build_scene("refraction", 128), 128)
cam = vrt.make_camera(W, H)
p = vrt.default_params(4, 4)


def timed(fn, frames, warm=300):
    fn(warm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    t0 = time.perf_counter()
    fn(frames)
    host = (time.perf_counter() - t0) * 1e3 / frames
    e1.record(main)
    torch.cuda.synchronize()
    return host, e0.elapsed_time(e1) / frames


for k in (1, 8):
    h = H // k

    def band(row0, rows, step, out, prev):
        ren.render_temporal_rows_async(cam, p, 1.0, row0, rows, step * k, prev.data_ptr(),
                                       out.data_ptr(), 0, 0, 0,
                                       torch.cuda.current_stream(dev).cuda_stream,
                                       pitch=row_pitch(out))

    t = FrameTiler(W, h, band, dev, dtype=torch.uint8, parts=1, gather=False, lanes=4,
                   independent=True)

    def tiler(n):
        for _ in range(n):
            t.frame()
        t.finish()

    streams = [torch.cuda.Stream(device=dev) for _ in range(4)]
    bufs = [torch.zeros((h, W, 4), dtype=torch.uint8, device=dev) for _ in range(4)]
    sptr = [s.cuda_stream for s in streams]
    bptr = [b.data_ptr() for b in bufs]
    st = {"f": 0}

    def raw(n):
        for s in streams:
            s.wait_stream(main)
        for _ in range(n):
            g = st["f"] % 4
            st["f"] += 1
            ren.render_temporal_rows_async(cam, p, 1.0, 0, h, k, bptr[g], bptr[g], 0, 0, 0, sptr[g],
                                           pitch=W)
        for s in streams:
            main.wait_stream(s)

    for name, fn in (("tiler", tiler), ("raw", raw)):
        hm, gm = timed(fn, 2000)
        print(f"k={k} {name:5s}: host {hm:.4f} ms/frame, GPU {gm:.4f} ms/frame", flush=True)

s = torch.cuda.Stream(device=dev)


def devf(n):
    s.wait_stream(main)
    for _ in range(n):
        ren.render_frame_device(cam, p, 1.0, s.cuda_stream)
    main.wait_stream(s)


hm, gm = timed(devf, 2000)
print(f"k=1 dev  : host {hm:.4f} ms/frame, GPU {gm:.4f} ms/frame", flush=True)
