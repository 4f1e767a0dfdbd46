#!/usr/bin/env python3
"""Experiment: hide the per-launch tail by rendering each frame as S interleaved-row parts on S
HIP streams (part s = rows s, s+S, ...; each part's temporal history is its own rows, so the
frame-to-frame dependency stays inside one stream). Reports ms per frame for S = 1, 2, 3, 4 over
K frames after warm-up, and checks the assembled frame equals the single-stream one.
Usage: python scripts/streams_exp.py [--config C3] [--frames 300] [--warmup 200]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import voxelraytracer_amd as vrt  # noqa: E402
from bench import CONFIGS  # noqa: E402


_STREAMS = []


def run(ren, cam, p, w, h, parts, frames, warmup):
    if os.environ.get("STREAMS_FRESH"):   # a new set of streams per run (the old behaviour)
        streams = [torch.cuda.Stream() for _ in range(parts)]
    else:                                 # one set of streams for the whole process
        while len(_STREAMS) < parts:
            _STREAMS.append(torch.cuda.Stream())
        streams = _STREAMS[:parts]
    rows = h // parts
    bufs = [torch.zeros((rows, w, 4), dtype=torch.uint8, device="cuda") for _ in range(parts)]
    main = torch.cuda.current_stream()

    def frame():
        for s in range(parts):
            ren.render_temporal_rows_async(cam, p, 1.0, s, rows, parts, bufs[s].data_ptr(),
                                           bufs[s].data_ptr(), stream=streams[s].cuda_stream)

    for _ in range(warmup):
        frame()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for st in streams:
        st.wait_event(e0)
    for _ in range(frames):
        frame()
    for st in streams:
        main.wait_stream(st)
    e1.record(main)
    torch.cuda.synchronize()
    img = torch.stack(bufs).permute(1, 0, 2, 3).reshape(h, w, 4).cpu().numpy()
    return e0.elapsed_time(e1) / frames, img


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C3")
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--parts", default="1,2,3,4,1,2")
    a = ap.parse_args()
    for cfg in a.configs.split(","):
        scene, n, w, h, R, T, _ = CONFIGS[cfg]
        with vrt.Renderer(0) as ren:
            ren.upload_volume(vrt.build_scene(scene, n), n)
            cam = vrt.make_camera(w, h)
            p = vrt.default_params(R, T)
            base = None
            for parts in (int(x) for x in a.parts.split(",")):
                if h % parts:
                    continue
                ms, img = run(ren, cam, p, w, h, parts, a.frames, a.warmup)
                same = True if base is None else bool(np.array_equal(img, base))
                base = img if base is None else base
                lib = os.path.basename(os.environ.get("VRT_LIB", "libvrt.so"))
                print(f"{cfg} {lib} parts={parts}: {ms:.4f} ms/frame  identical={same}",
                      flush=True)


if __name__ == "__main__":
    main()
