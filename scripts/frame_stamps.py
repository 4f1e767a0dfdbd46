#!/usr/bin/env python3
"""Where the fused frame's time goes (frame_kernel): per-wave timeline from the diagnostic build
(make variant NAME=stamps DEFS=-DVRT_STAMPS; run with VRT_LIB=build/variants/libvrt_stamps.so).

Each wave records s_memrealtime (100 MHz) at its start, after its certified phase, after the
completion counters and at its end, plus its deferred-pixel count, whether it rendered them in
place, drains its class's partial batch or belongs to the heavy-first pass, and the full queue
batches it owns. One band is rendered
alone a few times in the fused mode; the last launch's stamps are summarised.
Usage: VRT_LIB=... python scripts/frame_stamps.py --config C3 [--ranks 8 --rank R] [--mode 3]"""
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


def q(x, qs=(0.5, 0.9, 0.99, 1.0)):
    return {str(k): round(float(np.quantile(x, k)), 2) for k in qs} if len(x) else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--mode", type=int, default=3)
    ap.add_argument("--frames", type=int, default=6)
    args = ap.parse_args()
    lib = abi.load_library()
    if not hasattr(lib, "vrt_debug_stamps5"):
        sys.exit("VRT_LIB must point at the VRT_STAMPS diagnostic build")
    lib.vrt_debug_stamps5.restype = C.c_int
    lib.vrt_debug_stamps5.argtypes = [C.c_void_p, C.c_uint64]
    scene, n, w, h, R, T, _ = CONFIGS[args.config]
    row0, rows, step = (0, h, 1) if args.ranks == 1 else block_band_spec(args.rank, args.ranks, h, 16)
    block = 1 if args.ranks == 1 else 16
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    cam = vrt.make_camera(w, h)
    params = vrt.default_params(R, T)
    buf = torch.zeros((rows, w, 4), dtype=torch.uint8, device=dev)
    tiles = -(-w // 16) * -(-rows // 8)
    ord_q = -(-tiles // 32)
    waves = (8 * ord_q + tiles) * 2
    with vrt.Renderer(0) as ren:
        ren.build_scene_device(scene, n)
        ren.set_exact_pass(args.mode)
        for _ in range(args.frames):
            ren.render_temporal_rows_async(cam, params, 1.0, row0, rows, step, buf.data_ptr(), buf.data_ptr(),
                                           stream=st, row_block=block)
            torch.cuda.synchronize()
        s = np.zeros((waves, 8), np.uint64)
        assert lib.vrt_debug_stamps5(s.ctypes.data, s.size) == 0
    busy = np.nonzero(s[:, 0])[0]
    s = s[busy]
    t0 = s[:, 0].min()
    us = lambda c: (s[:, c] - t0).astype(np.float64) * 10e-3   # noqa: E731
    start, cert, done, end = us(0), us(1), us(2), us(3)
    info = s[:, 4].astype(np.int64)
    cnt, inplace, setf, heavy = info & 0xFF, (info >> 8) & 1, (info >> 9) & 1, (info >> 10) & 1
    claims = s[:, 5].astype(np.int64)
    exact = (inplace == 1) | (claims > 0) | (setf == 1)
    out = {"config": args.config, "band": [row0, rows, step, block], "mode": args.mode,
           "waves": int(len(busy)), "span_us": round(float(end.max()), 2),
           "last_certified_phase_end_us": round(float(cert.max()), 2),
           "cert_phase_us": q(cert - start), "counter_phase_us": q(done - cert),
           "heavy_pass": {"waves": int(heavy.sum()),
                          "cert_end_us": round(float(cert[heavy == 1].max()), 2) if heavy.any() else None},
           "class_drains_at_us": sorted(round(float(x), 2) for x in done[setf == 1]),
           "appending_waves": int(((cnt > 0) & (inplace == 0)).sum()), "appended": int(cnt[inplace == 0].sum()),
           "in_place_waves": int(inplace.sum()), "in_place_pixels": int(cnt[inplace == 1].sum()),
           "owned_batches": int(claims.sum()),
           "exact_waves": {"n": int(exact.sum()), "exact_phase_us": q(end[exact] - done[exact]),
                           "start_of_exact_us": q(done[exact]), "end_us": q(end[exact])},
           "other_waves_end_us": q(end[~exact])}
    order = np.argsort(-end)[:10]
    out["latest"] = [{"end_us": round(float(end[i]), 2), "start_us": round(float(start[i]), 2),
                      "cert_end_us": round(float(cert[i]), 2), "exact_from_us": round(float(done[i]), 2),
                      "cnt": int(cnt[i]), "in_place": bool(inplace[i]), "batches": int(claims[i]),
                      "class_drain": bool(setf[i])} for i in order]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
