"""Strong-scaling rehearsal with frames in flight, on one GPU.

For k = 1, 2, 4, 8 this renders GPU 0's cyclic band of the frame (rows 0, k, 2k, ...) with the
fused temporal filter at u_Alpha = 1, the slider default: a frame then does not read its history,
so consecutive frames are independent. Frames rotate over G "lanes"; a lane is P part streams
(the band's P interleaved row parts) and its own output buffer, so frame f renders into
ring[f % G] on lane f % G and frames f, f+1, ..., f+G-1 are in flight at once: the light waves of
the next frames fill the wave slots that one frame's long exact-path waves hold. G = 1, P = 2 is
the round-2 scheme (scripts/diag/strong_bands.py).

Prints ms per frame in the steady state (K frames after W warm-ups, one event pair) and checks
that every lane's last frame is bit-identical to one frame rendered alone.
Usage: python scripts/diag/strong_pipe.py [CFG ...] [--lanes 1x2,2x2,3x2,4x1,4x2,8x1]
"""
import argparse
import os
import sys

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")   # before HIP initialises

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import voxelraytracer_amd as vrt  # noqa: E402

CONFIGS = {  # scene, N, W, H, (R, T)
    "C1": ("glass_cube", 128, 1920, 1080, (1, 2)),
    "C2": ("terrain", 128, 1920, 1080, (4, 2)),
    "C3": ("refraction", 128, 1920, 1080, (4, 4)),
    "C4": ("terrain", 512, 3840, 2160, (4, 2)),
}


def run(r, cam, p, h, w, k, lanes, parts, warm, frames):
    plan, _ = vrt.band_plan(h, k, parts)
    specs = [plan[(0, q)] for q in range(parts)]   # (row0, rows, row_step, band_row0)
    rows = sum(x[1] for x in specs)
    ring = [torch.zeros((rows, w, 4), dtype=torch.uint8, device="cuda") for _ in range(lanes)]
    streams = [[torch.cuda.Stream() for _ in range(parts)] for _ in range(lanes)]
    main = torch.cuda.current_stream()
    state = {"f": 0}

    def frames_(count):
        for ln in streams:
            for st in ln:
                st.wait_stream(main)
        for _ in range(count):
            g = state["f"] % lanes
            state["f"] += 1
            buf = ring[g]
            for st, (row0, prow, step, brow0) in zip(streams[g], specs):
                view = buf[brow0:]
                r.render_temporal_rows_async(cam, p, 1.0, row0, prow, step, view.data_ptr(),
                                             view.data_ptr(), stream=st.cuda_stream,
                                             pitch=parts * w)
        for ln in streams:
            for st in ln:
                main.wait_stream(st)

    frames_(warm)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    frames_(frames)
    e1.record(main)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / frames
    # reference: the same band alone, one launch, exact STATS instance (counters on)
    ref = torch.zeros((rows, w, 4), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(len(vrt.COUNTER_NAMES), dtype=torch.int64, device="cuda")
    r.render_temporal_rows_async(cam, p, 1.0, 0, rows, k, ref.data_ptr(), ref.data_ptr(),
                                 d_counters=cnt.data_ptr(), stream=main.cuda_stream)
    torch.cuda.synchronize()
    bad = sum(int((b != ref).sum().item()) for b in ring)
    return ms, rows, bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfgs", nargs="*", default=["C3", "C4"])
    ap.add_argument("--lanes", default="1x2,2x2,3x2,4x2,4x1,6x1,8x1")
    ap.add_argument("--ks", default="1,2,4,8")
    ap.add_argument("--warm", type=int, default=100)
    ap.add_argument("--frames", type=int, default=400)
    a = ap.parse_args()
    modes = [tuple(int(v) for v in m.split("x")) for m in a.lanes.split(",")]
    ks = [int(v) for v in a.ks.split(",")]
    for name in a.cfgs:
        scene, n, w, h, (rr, tt) = CONFIGS[name]
        with vrt.Renderer(0) as r:
            r.upload_volume(vrt.build_scene(scene, n), n)
            cam = vrt.make_camera(w, h)
            p = vrt.default_params(rr, tt)
            base = {}
            for (g, pp) in modes:
                for k in ks:
                    ms, rows, bad = run(r, cam, p, h, w, k, g, pp, a.warm, a.frames)
                    base.setdefault((g, pp), {})[k] = ms
                    t1 = base[(1, 2)][1] if (1, 2) in base and 1 in base[(1, 2)] else None
                    sp = f"{t1 / ms:.2f}x vs 1x2 k=1" if t1 else ""
                    own = base[(g, pp)].get(1)
                    print(f"{name} lanes {g}x{pp} k={k}: band {rows} rows: {ms:.4f} ms/frame  "
                          f"{sp}  self {own / ms:.2f}x  mismatched {bad}", flush=True)


if __name__ == "__main__":
    main()
