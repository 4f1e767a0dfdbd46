#!/usr/bin/env python3
"""Where the deferred exact pass's time goes: per-wave timeline of exact_pass_kernel from the
diagnostic build (make variant NAME=stamps DEFS=-DVRT_STAMPS; run with
VRT_LIB=build/variants/libvrt_stamps.so).

Each busy exact-pass workgroup (one wave) records s_memrealtime (100 MHz) at start and end, its
pixels (dense chunk or compact batch), and exact_pixel's stamps after the primary trace (exact
primary walk + its shadow) and after the bounce stack. One band (the whole frame, or rank R's
16-row block band of a K-way split) is rendered alone a few times with the exact pass forced;
the last launch's stamps are summarised: kernel span, wave-duration quantiles, and the phase split
of the longest waves. Usage: VRT_LIB=... python scripts/exact_stamps.py --config C3 [--ranks 8]
"""
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
from voxelraytracer_amd.tiles import block_band_spec  # noqa: E402
from bench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--top", type=int, default=12)
    args = ap.parse_args()
    lib = abi.load_library()
    if not hasattr(lib, "vrt_debug_stamps4"):
        sys.exit("VRT_LIB must point at the VRT_STAMPS diagnostic build")
    for f in ("vrt_debug_stamps3", "vrt_debug_stamps4"):
        getattr(lib, f).restype = C.c_int
        getattr(lib, f).argtypes = [C.c_void_p, C.c_uint64]
    scene, n, w, h, R, T, _ = CONFIGS[args.config]
    row0, rows, step = (0, h, 1) if args.ranks == 1 else block_band_spec(args.rank, args.ranks, h, 16)
    block = 1 if args.ranks == 1 else 16
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    cam = vrt.make_camera(w, h)
    params = vrt.default_params(R, T)
    buf = torch.zeros((rows, w, 4), dtype=torch.uint8, device=dev)
    with vrt.Renderer(0) as ren:
        ren.build_scene_device(scene, n)
        ren.set_exact_pass(2)
        for _ in range(6):
            ren.render_temporal_rows_async(cam, params, 1.0, row0, rows, step, buf.data_ptr(), buf.data_ptr(),
                                           stream=st, row_block=block)
            torch.cuda.synchronize()
        tiles = -(-w // 16) * -(-rows // 8)
        grid = max(64, tiles * 2 // 8)
        s4 = np.zeros((grid, 4), np.uint64)
        s3 = np.zeros((2 * grid, 2), np.uint64)
        assert lib.vrt_debug_stamps4(s4.ctypes.data, s4.size) == 0
        assert lib.vrt_debug_stamps3(s3.ctypes.data, s3.size) == 0
    busy = np.nonzero(s4[:, 0])[0]
    t0 = s4[busy, 0].min()
    start = (s4[busy, 0] - t0).astype(np.float64) * 10e-3   # us
    end = (s4[busy, 1] - t0).astype(np.float64) * 10e-3
    dur = end - start
    px = (s4[busy, 3] & np.uint64(0xFFFF)).astype(np.int64)
    dense = (s4[busy, 3] >> np.uint64(16)).astype(np.int64)
    prim = s3[2 * busy, 0]
    bounce = s3[2 * busy, 1]
    out = {"config": args.config, "band": [row0, rows, step, block], "busy_waves": int(len(busy)),
           "span_us": round(float(end.max()), 2),
           "wave_us_quantiles": {q: round(float(np.quantile(dur, q)), 2) for q in (0.5, 0.9, 0.99, 1.0)},
           "dense_waves": int((dense > 0).sum()), "pixels": int(px.sum()), "longest": []}
    for kind, m in (("dense", dense > 0), ("sparse", dense == 0)):
        if m.any():
            pr = np.where(prim[m] >= s4[busy[m], 0], (prim[m] - s4[busy[m], 0]).astype(np.float64) * 10e-3, np.nan)
            out[kind] = {"waves": int(m.sum()),
                         "wave_us": {q: round(float(np.quantile(dur[m], q)), 2) for q in (0.5, 0.9, 1.0)},
                         "primary_trace_us": {q: round(float(np.nanquantile(pr, q)), 2) for q in (0.5, 0.9, 1.0)}}
    for i in np.argsort(-dur)[:args.top]:
        p = (float(prim[i] - s4[busy[i], 0]) * 10e-3) if prim[i] >= s4[busy[i], 0] else None
        b = (float(bounce[i] - prim[i]) * 10e-3) if bounce[i] >= prim[i] > 0 else None
        out["longest"].append({"wave": int(busy[i]), "start_us": round(start[i], 2), "dur_us": round(dur[i], 2),
                               "pixels": int(px[i]), "dense": bool(dense[i]),
                               "primary_trace_us": None if p is None else round(p, 2),
                               "bounce_stack_us": None if b is None else round(b, 2)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
