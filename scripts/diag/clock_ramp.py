"""Why the first frames of a fresh process are slow: per-group GPU time of C3 frames (bench's
FrameTiler, two parts) with no host sync between groups, after different preludes.
  plain  : frames right after setup (as bench.py does)
  spin   : ~SPIN_MS of unrelated GPU work (bf16 matmuls) first
  render : ~SPIN_MS of exact-instance renders first (heavier per launch than the frames)
Usage: python scripts/diag/clock_ramp.py MODE [SPIN_MS]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import voxelraytracer_amd as vrt  # noqa: E402
from voxelraytracer_amd.tiles import FrameTiler, row_pitch  # noqa: E402

mode = sys.argv[1]
spin_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
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
if mode == "spin":
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < spin_ms:
        for _ in range(8):
            a = (a @ a).clamp_(-1, 1)
        torch.cuda.synchronize()
elif mode == "render":
    out = torch.zeros((1080, 1920, 4), dtype=torch.float32, device=dev)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < spin_ms:
        ren.render_rows_async(cam, p, 0, 1080, 1, out.data_ptr(), 0, 0, s.cuda_stream)
        torch.cuda.synchronize()
import glob
import threading
clk = []
stop = []
files = sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_sclk"))


def sample():   # the engine clock's current DPM level while the frames run (sysfs, if readable)
    t0 = time.perf_counter()
    while not stop:
        for f in files[:1]:
            try:
                cur = [l for l in open(f).read().splitlines() if "*" in l]
                clk.append((round((time.perf_counter() - t0) * 1e3, 1), cur[0].split(":")[1].strip() if cur else "?"))
            except OSError as e:
                clk.append((0, str(e)))
                stop.append(1)
        time.sleep(0.002)


th = threading.Thread(target=sample, daemon=True)
th.start()
evs = []
for g in range(40):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(10):
        t.frame()
    t.finish()
    e1.record(s)
    evs.append((e0, e1))
torch.cuda.synchronize()
stop.append(1)
th.join()
ms = [a.elapsed_time(b) / 10 for a, b in evs]
print("sclk samples (ms, level):", files[:1], clk[:: max(1, len(clk) // 30)])
print(f"{mode:6s} ms/frame per group of 10:", " ".join(f"{x:.4f}" for x in ms), flush=True)
