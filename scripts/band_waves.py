#!/usr/bin/env python3
"""Longest waves of one block-cyclic band rendered alone, in lane (diagnostic build
make variant NAME=stamps DEFS=-DVRT_STAMPS; run with VRT_LIB=build/diag/libvrt_stamps.so).

Renders rank R's band of a K-way split (blocks of B rows) with the exact path in lane and no tile
order, the way bench.py's 8-way C3 bands run, and prints the wave-duration quantiles, the span,
and the longest waves with their frame rows / pixel columns, the exact lanes of the wave and the
split of its time into certified attempt, exact primary trace and bounce stacks. A band whose
frames-in-flight rate is latency-bound (bench.py --rehearse-rank) shows here as a longer longest
wave. Usage: VRT_LIB=... python scripts/band_waves.py --config C3 --ranks 8 --rank 4 --block 8"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import voxelraytracer_amd as vrt  # noqa: E402
from voxelraytracer_amd import abi  # noqa: E402
from voxelraytracer_amd.tiles import block_band_spec, band_frame_rows  # noqa: E402
from bench import CONFIGS  # noqa: E402


def stamps(lib, name, rows_n, cols):
    f = getattr(lib, name)
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_uint64]
    a = np.zeros((rows_n, cols), dtype=np.uint64)
    assert f(a.ctypes.data, a.size) == 0
    return a


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--block", type=int, default=16)
    ap.add_argument("--top", type=int, default=8)
    args = ap.parse_args()
    lib = abi.load_library()
    if not hasattr(lib, "vrt_debug_stamps3"):
        sys.exit("VRT_LIB must point at the VRT_STAMPS diagnostic build")
    scene, n, w, h, R, T, _ = CONFIGS[args.config]
    row0, rows, step = block_band_spec(args.rank, args.ranks, h, args.block)
    frow = band_frame_rows(row0, rows, step, args.block).numpy()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    cam = vrt.make_camera(w, h)
    params = vrt.default_params(R, T)
    buf = torch.zeros((rows, w), dtype=torch.int32, device=dev)
    with vrt.Renderer(0) as ren:
        ren.build_scene_device(scene, n)
        ren.set_exact_pass(0)
        ren.set_tile_order(0)
        for _ in range(6):
            ren.render_temporal_rows_async(cam, params, 1.0, row0, rows, step, buf.data_ptr(), buf.data_ptr(),
                                           stream=st, row_block=args.block)
            torch.cuda.synchronize()
    tiles_x = -(-w // 16)
    tiles = tiles_x * -(-rows // 8)
    waves = tiles * 2
    s1 = stamps(lib, "vrt_debug_stamps", waves, 3)
    s2 = stamps(lib, "vrt_debug_stamps2", waves, 2)
    s3 = stamps(lib, "vrt_debug_stamps3", waves, 2)
    t0 = s1[:, 0].min()
    start = (s1[:, 0] - t0) * 10.0 / 1e3   # us (100 MHz)
    end = (s1[:, 1] - t0) * 10.0 / 1e3
    dur = end - start
    order = np.argsort(-dur)[:args.top]
    longest = []
    for wv in order:
        tile, sub = divmod(int(wv), 2)
        ty, tx = divmod(tile, tiles_x)
        band_row = ty * 8
        cert_us = (float(s2[wv, 0]) - float(s1[wv, 0])) * 10.0 / 1e3 if s2[wv, 0] else None
        prim_us = (float(s3[wv, 0]) - float(s2[wv, 0])) * 10.0 / 1e3 if s3[wv, 0] and s2[wv, 0] else None
        stack_us = (float(s3[wv, 1]) - float(s3[wv, 0])) * 10.0 / 1e3 if s3[wv, 1] and s3[wv, 0] else None
        longest.append({"wave": int(wv), "frame_rows": [int(frow[band_row]), int(frow[min(band_row + 7, rows - 1)])],
                        "px": [tx * 16 + sub * 8, tx * 16 + sub * 8 + 7], "start_us": round(float(start[wv]), 2),
                        "dur_us": round(float(dur[wv]), 2), "exact_lanes": int(s2[wv, 1]),
                        "cert_us": cert_us and round(cert_us, 2), "primary_us": prim_us and round(prim_us, 2),
                        "stack_us": stack_us and round(stack_us, 2)})
    q = np.quantile(dur, [0.5, 0.9, 0.99, 1.0])
    print(json.dumps({"config": args.config, "ranks": args.ranks, "rank": args.rank, "block": args.block,
                      "rows": int(rows), "waves": int(waves), "span_us": round(float(end.max()), 2),
                      "wave_us_quantiles": dict(zip(["0.5", "0.9", "0.99", "1.0"], [round(float(x), 2) for x in q])),
                      "exact_waves": int((s2[:, 1] > 0).sum()), "longest": longest}, indent=1))


if __name__ == "__main__":
    main()
