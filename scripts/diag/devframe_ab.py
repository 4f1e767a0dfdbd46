"""GPU time per frame of device-output frames (vrt_render_frame_device, C3, four lanes) against
the bench's lean band launches, for the product library and the diagnostic VRT_DEV_* variants
(build/variants): what the library's per-frame ordering (the caller stream's wait for each frame,
the consumption wait for the ring slot) costs. Each library runs in its own process (VRT_LIB).
Usage: python scripts/diag/devframe_ab.py [frames]"""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r"""
import os, sys, time
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import torch
sys.path.insert(0, %r)
import voxelraytracer_amd as vrt
n = int(sys.argv[1])
dev = torch.device("cuda", 0)
main = torch.cuda.current_stream(dev)
r = vrt.Renderer(0)
r.upload_volume(vrt.build_scene("refraction", 128), 128)
cam = vrt.make_camera(1920, 1080)
p = vrt.default_params(4, 4)
s = torch.cuda.Stream(device=dev)
def run(k):
    s.wait_stream(main)
    for _ in range(k):
        r.render_frame_device(cam, p, 1.0, s.cuda_stream)
    main.wait_stream(s)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.2:
    run(50); torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(main); run(n); e1.record(main); torch.cuda.synchronize()
print("%%.4f" %% (e0.elapsed_time(e1) / n))
""" % ROOT


def main():
    n = sys.argv[1] if len(sys.argv) > 1 else "1000"
    libs = [("product", None)] + [(os.path.basename(l)[7:-3], l) for l in
                                  sorted(glob.glob(os.path.join(ROOT, "build", "variants", "libvrt_*.so")))]
    for rnd in range(2):
        for name, lib in libs:
            env = dict(os.environ)
            env.pop("VRT_LIB", None)
            if lib:
                env["VRT_LIB"] = lib
            out = subprocess.run([sys.executable, "-c", CHILD, n], capture_output=True, text=True,
                                 env=env, timeout=120)
            print(f"round {rnd} {name:10s} device frames: {out.stdout.strip() or out.stderr[-300:]} ms/frame",
                  flush=True)


if __name__ == "__main__":
    main()
