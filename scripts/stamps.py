#!/usr/bin/env python3
"""Wave timeline of one render from the diagnostic build (make variant NAME=stamps
DEFS=-DVRT_STAMPS; run with VRT_LIB=build/variants/libvrt_stamps.so).

Each wave of render_kernel records s_memrealtime (100 MHz) at entry and exit plus its HW_ID /
XCC_ID. Prints, per config: the kernel span, wave-duration quantiles, the busy fraction of the
wave slots (sum of wave durations / (span x slots)), how the span splits into ramp (until every
slot has started a wave), steady state and tail (after the last wave started), and the per-XCD
finish times. Optional --save writes the raw stamps (npz) for plotting.
Usage: VRT_LIB=build/variants/libvrt_stamps.so python scripts/stamps.py [--configs C3] [--save d]
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
from bench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C3")
    ap.add_argument("--wg-waves", type=int, default=2)
    ap.add_argument("--slots", type=int, default=256 * 4 * 6, help="wave slots (CUs*SIMDs*occupancy)")
    ap.add_argument("--save", default="")
    ap.add_argument("--tile-order", action="store_true",
                    help="keep the heavy-first tile order on (grid = 8*q + tiles slots; empty slots "
                         "leave no stamps and are dropped)")
    ap.add_argument("--band", default="", help="ROW0,ROWS: also time that band alone (few waves, "
                    "each alone on its SIMD) against the same tiles inside the full frame")
    args = ap.parse_args()
    lib = abi.load_library()
    if not hasattr(lib, "vrt_debug_stamps"):
        sys.exit("VRT_LIB must point at the VRT_STAMPS diagnostic build")
    lib.vrt_debug_stamps.restype = C.c_int
    lib.vrt_debug_stamps.argtypes = [C.c_void_p, C.c_uint64]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    report = {}
    for cfg in args.configs.split(","):
        scene, n, w, h, R, T, _ = CONFIGS[cfg]
        cam = vrt.make_camera(w, h)
        params = vrt.default_params(R, T)
        vox = torch.from_numpy(vrt.build_scene(scene, n)).to(dev)
        out = torch.empty((h, w, 4), dtype=torch.float32, device=dev)
        with vrt.Renderer(0) as ren:
            ren.upload_volume_device(vox.data_ptr(), n, stream.cuda_stream)
            # stamps are indexed by workgroup: the heavy-first tile order's two-pass grid leaves
            # slots without stamps (their tile is rendered by the other pass), so time dispatch order
            ren.set_tile_order(args.tile_order)
            for _ in range(5):   # warm; the stamps of the last launch are kept
                ren.render_rows_async(cam, params, 0, h, 1, out.data_ptr(), 0, 0, stream.cuda_stream)
            torch.cuda.synchronize()
        tw, th = (16, 16) if args.wg_waves == 4 else ((16, 8) if args.wg_waves == 2 else (8, 8))
        waves = ((w + tw - 1) // tw) * ((h + th - 1) // th) * args.wg_waves
        tiles = waves // args.wg_waves
        slots = tiles + (8 * ((tiles + 31) // 32) if args.tile_order else 0)  # VRT_ORD_DIV 4
        st = np.zeros((slots * args.wg_waves, 3), dtype=np.uint64)
        assert lib.vrt_debug_stamps(st.ctypes.data, st.size) == 0
        keep = st[:, 0] != 0
        wave_index = np.nonzero(keep)[0] if args.tile_order else np.arange(len(st))
        if args.tile_order:
            st = st[keep]
            waves = len(st)
        t0 = st[:, 0].min()
        start = (st[:, 0] - t0).astype(np.float64) * 10.0   # ns (100 MHz)
        end = (st[:, 1] - t0).astype(np.float64) * 10.0
        dur = end - start
        span = end.max()
        xcc = (st[:, 2] >> np.uint64(32)).astype(np.int64) & 0xF
        order = np.sort(start)
        ramp = order[min(args.slots, waves) - 1]          # all slots have started a wave
        last_start = order[-1]
        q = np.quantile(dur, [0.0, 0.1, 0.5, 0.9, 0.99, 1.0])
        r = dict(
            waves=int(waves), span_us=span / 1e3,
            wave_us_quantiles=dict(zip(["min", "p10", "p50", "p90", "p99", "max"],
                                       [round(x / 1e3, 2) for x in q])),
            slot_busy_frac=float(dur.sum() / (span * args.slots)),
            ramp_us=ramp / 1e3, last_start_us=last_start / 1e3,
            tail_us=(span - last_start) / 1e3,
            xcd_finish_us={int(x): round(float(end[xcc == x].max()) / 1e3, 1)
                           for x in np.unique(xcc)},
            xcd_wave_ms_sum={int(x): round(float(dur[xcc == x].sum()) / 1e6, 2)
                             for x in np.unique(xcc)},
        )
        # busy slots over time (10 bins): how many waves are resident
        edges = np.linspace(0, span, 11)
        mids = (edges[:-1] + edges[1:]) / 2
        r["resident_waves_over_time"] = [int(((start <= m) & (end > m)).sum()) for m in mids]
        if args.band:
            b0, brows = (int(x) for x in args.band.split(","))
            tile_row = lambda wl: (wl // args.wg_waves // ((w + tw - 1) // tw)) * (th // 8) + \
                ((wl % args.wg_waves) >> 1)
            full_rows = tile_row(np.arange(waves))
            sel = (full_rows >= b0 // 8) & (full_rows < (b0 + brows) // 8)
            with vrt.Renderer(0) as ren:
                ren.upload_volume_device(vox.data_ptr(), n, stream.cuda_stream)
                ren.set_tile_order(False)
                for _ in range(3):
                    ren.render_rows_async(cam, params, b0, brows, 1, out.data_ptr(), 0, 0,
                                          stream.cuda_stream)
                torch.cuda.synchronize()
            bw = ((w + tw - 1) // tw) * ((brows + th - 1) // th) * args.wg_waves
            sb = np.zeros((bw, 3), dtype=np.uint64)
            assert lib.vrt_debug_stamps(sb.ctypes.data, sb.size) == 0
            db = (sb[:, 1] - sb[:, 0]).astype(np.float64) * 10.0
            r["band"] = dict(rows=[b0, brows], waves_alone=int(bw),
                             mean_wave_us_alone=float(db.mean() / 1e3),
                             mean_wave_us_in_full_frame=float(dur[sel].mean() / 1e3),
                             span_us_alone=float((sb[:, 1].max() - sb[:, 0].min()) * 10.0 / 1e3))
        report[cfg] = r
        print(cfg, json.dumps(r))
        if args.save:
            os.makedirs(args.save, exist_ok=True)
            extra = {}
            if hasattr(lib, "vrt_debug_stamps2"):  # {time after the certified attempt, exact lanes}
                lib.vrt_debug_stamps2.restype = C.c_int
                lib.vrt_debug_stamps2.argtypes = [C.c_void_p, C.c_uint64]
                st2 = np.zeros((len(keep), 2), dtype=np.uint64)
                assert lib.vrt_debug_stamps2(st2.ctypes.data, st2.size) == 0
                st2 = st2[keep] if args.tile_order else st2[:waves]
                extra["stamps2"] = st2
            if hasattr(lib, "vrt_debug_stamps3"):  # {after the exact primary trace, after the stacks}
                lib.vrt_debug_stamps3.restype = C.c_int
                lib.vrt_debug_stamps3.argtypes = [C.c_void_p, C.c_uint64]
                st3 = np.zeros((len(keep), 2), dtype=np.uint64)
                assert lib.vrt_debug_stamps3(st3.ctypes.data, st3.size) == 0
                st3 = st3[keep] if args.tile_order else st3[:waves]
                extra["stamps3"] = st3
            np.savez_compressed(os.path.join(args.save, f"stamps_{cfg}.npz"), stamps=st,
                                wave_index=wave_index, **extra)
    return report


if __name__ == "__main__":
    main()
