"""Strong-scaling rehearsal on one GPU: the band one GPU of a k-GPU split renders per frame.

For k = 1, 2, 4, 8 this renders GPU 0's cyclic band of the frame (rows 0, k, 2k, ...; as two
interleaved parts on two streams, vrt_band_plan) with the fused temporal filter, in place, and times
it over many frames. That is the per-frame compute of one GPU in the library's k-device frame
(vrt_render_frame_device) and in bench.py --scaling strong; the RGBA8 gather of the other bands
(pipelined under the next frame's render) is not included.
Usage: python scripts/diag/strong_bands.py [CFG ...]   (default C4 C3)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import voxelraytracer_amd as vrt  # noqa: E402

CONFIGS = {  # scene, N, W, H, (R, T)
    "C1": ("glass_cube", 128, 1920, 1080, (1, 2)),
    "C2": ("terrain", 128, 1920, 1080, (4, 2)),
    "C3": ("refraction", 128, 1920, 1080, (4, 4)),
    "C4": ("terrain", 512, 3840, 2160, (4, 2)),
}


def band_ms(r, cam, p, h, w, k, warm=200, frames=400):
    plan, _ = vrt.band_plan(h, k, 2)
    parts = [plan[(0, q)] for q in range(2)]   # GPU 0's two parts: (row0, rows, row_step, band_row0)
    rows = sum(x[1] for x in parts)
    buf = torch.zeros((rows, w, 4), dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    main = torch.cuda.current_stream()

    def frames_(count):   # parts run on their own streams (like bench.py's FrameTiler): no join
        for st in streams:
            st.wait_stream(main)
        for _ in range(count):
            for st, (row0, prow, step, brow0) in zip(streams, parts):
                view = buf[brow0:]   # band rows brow0, brow0 + 2, ...: pitch 2 rows
                r.render_temporal_rows_async(cam, p, 1.0, row0, prow, step, view.data_ptr(),
                                             view.data_ptr(), stream=st.cuda_stream, pitch=2 * w)
        for st in streams:
            main.wait_stream(st)

    frames_(warm)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    frames_(frames)
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / frames, rows


def main():
    cfgs = sys.argv[1:] or ["C4", "C3"]
    for name in cfgs:
        scene, n, w, h, (rr, tt) = CONFIGS[name]
        with vrt.Renderer(0) as r:
            r.upload_volume(vrt.build_scene(scene, n), n)
            cam = vrt.make_camera(w, h)
            p = vrt.default_params(rr, tt)
            t1 = None
            for k in (1, 2, 4, 8):
                ms, rows = band_ms(r, cam, p, h, w, k)
                t1 = t1 or ms
                print(f"{name} k={k}: GPU 0 band {rows} rows x {w}: {ms:.4f} ms/frame, "
                      f"speed-up if every band took as long {t1 / ms:.2f}x (ideal {k}x)", flush=True)


if __name__ == "__main__":
    main()
