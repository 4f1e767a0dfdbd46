"""The fresh-process ramp of bench.py's frame time (driver's --steps 20 --warmup 5 vs the settled
500/200 run): per-group GPU time of C3 frames through bench.py's FrameTiler (4 lanes) from the
first frame on, with the DPM levels of every card's engine / memory / fabric / SoC clocks and
gpu_busy_percent sampled from sysfs while they run (the busy card is the one whose load moves).
Usage: python scripts/diag/clock_ramp2.py [GROUPS] [FRAMES_PER_GROUP] [PRELUDE_MS]"""
import glob
import os
import sys
import threading
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import voxelraytracer_amd as vrt  # noqa: E402
from voxelraytracer_amd.tiles import FrameTiler, row_pitch  # noqa: E402

groups = int(sys.argv[1]) if len(sys.argv) > 1 else 60
per = int(sys.argv[2]) if len(sys.argv) > 2 else 20
prelude_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
dev = torch.device("cuda", 0)
torch.cuda.set_stream(torch.cuda.Stream(device=dev))
s = torch.cuda.current_stream(dev)
props = torch.cuda.get_device_properties(0)
print("device:", {k: getattr(props, k) for k in dir(props) if k.startswith("pci") or k in ("name", "uuid")})
ren = vrt.Renderer(0)
ren.upload_volume(vrt.build_scene("refraction", 128), 128)
cam = vrt.make_camera(1920, 1080)
p = vrt.default_params(4, 4)


def band(row0, rows, step, out, prev):
    sp = torch.cuda.current_stream(dev).cuda_stream
    ren.render_temporal_rows_async(cam, p, 1.0, row0, rows, step, prev.data_ptr(), out.data_ptr(),
                                   0, 0, 0, sp, pitch=row_pitch(out))


t = FrameTiler(1920, 1080, band, dev, dtype=torch.uint8, parts=1, gather=False, lanes=4,
               independent=True)
torch.cuda.synchronize()
cards = sorted(glob.glob("/sys/class/drm/card*/device"))
kinds = ["pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk", "pp_dpm_socclk"]
samples = []
stop = []


def cur_level(path):
    try:
        for line in open(path).read().splitlines():
            if "*" in line:
                return line.split(":")[1].replace("*", "").strip()
    except OSError:
        return None
    return "?"


def busy(path):
    try:
        return open(path).read().strip()
    except OSError:
        return None


def sample():
    t0 = time.perf_counter()
    while not stop:
        row = [round((time.perf_counter() - t0) * 1e3, 1)]
        for c in cards:
            row.append((os.path.basename(os.path.dirname(c)), busy(c + "/gpu_busy_percent"),
                        *[cur_level(f"{c}/{k}") for k in kinds]))
        samples.append(row)
        time.sleep(0.003)


th = threading.Thread(target=sample, daemon=True)
th.start()
time.sleep(0.05)
if prelude_ms > 0:   # the same frames for prelude_ms first, untimed
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < prelude_ms:
        for _ in range(20):
            t.frame()
        t.finish()
        torch.cuda.synchronize()
evs = []
for g in range(groups):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(per):
        t.frame()
    t.finish()
    e1.record(s)
    evs.append((e0, e1))
torch.cuda.synchronize()
time.sleep(0.05)
stop.append(1)
th.join()
ms = [a.elapsed_time(b) / per for a, b in evs]
print(f"prelude {prelude_ms} ms; ms/frame per group of {per}:", " ".join(f"{x:.4f}" for x in ms), flush=True)
# cards whose busy percent or clocks change
for ci, c in enumerate(cards):
    vals = [r[1 + ci] for r in samples]
    if len(set(v[1] for v in vals)) > 1 or len(set(v[2] for v in vals)) > 1:
        step = max(1, len(samples) // 40)
        print(os.path.basename(os.path.dirname(c)), "(t ms, busy%, sclk, mclk, fclk, socclk):")
        for r in samples[::step]:
            v = r[1 + ci]
            print("  ", r[0], v[1:], flush=True)
