#!/usr/bin/env python3
"""Interleaved in-process A/B of kernel variants (build/variants/libvrt_*.so + the default lib).

Each library is loaded as its own ctypes handle (RTLD_LOCAL); every round renders each config
once per variant in turn, so clock/thermal drift hits all variants alike. Prints the median and
min kernel ms per (variant, config) and checks that all variants agree bit-exactly on the image.
Each timed sample is --batch back-to-back launches (per-launch mean), which averages out the
launch-to-launch jitter of single-event timings.
Usage: python scripts/ab.py [--rounds 10] [--batch 8] [--configs C1,C2,C3]
"""
import argparse
import ctypes as C
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime: torch's)

import voxelraytracer_amd as vrt  # noqa: E402
from voxelraytracer_amd import abi  # noqa: E402
from bench import CONFIGS  # noqa: E402


def load(path):
    lib = C.CDLL(path)
    for name, (res, args) in abi.SIGNATURES.items():
        if not hasattr(lib, name):   # older variant builds may lack newer diagnostic symbols
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--configs", default="C1,C2,C3")
    ap.add_argument("--batch", type=int, default=8,
                    help="back-to-back launches per timed sample (ms reported per launch)")
    args = ap.parse_args()
    libs = {"base": abi.LIB_PATH}
    for p in sorted(glob.glob(os.path.join(ROOT, "build", "variants", "libvrt_*.so"))):
        libs[os.path.basename(p)[7:-3]] = p
    handles = {}
    for name, path in libs.items():
        L = load(path)
        h = C.c_void_p()
        assert L.vrt_create(1, C.byref(h)) == 0
        handles[name] = (L, h)
    res = {}
    for cfg in args.configs.split(","):
        scene, n, w, hgt, R, T, _ = CONFIGS[cfg]
        vox = vrt.build_scene(scene, n)
        cam = vrt.make_camera(w, hgt)
        p = vrt.default_params(R, T)
        vol = abi.Volume(vox.ctypes.data_as(C.POINTER(C.c_uint8)), n)  # noqa
        for L, h in handles.values():
            assert L.vrt_upload_volume(h, C.byref(vol)) == 0
        imgs = {}
        times = {k: [] for k in handles}
        stream = torch.cuda.current_stream()
        # the bench's output: RGB8 store + temporal filter (alpha 1), in place, one launch
        outs = {k: torch.zeros((hgt, w, 4), dtype=torch.uint8, device="cuda") for k in handles}
        for r in range(args.rounds + 2):
            for name, (L, h) in handles.items():
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                nb = 1 if r == 0 else args.batch
                e0.record(stream)
                for _ in range(nb):
                    d = outs[name].data_ptr()
                    rc = L.vrt_render_temporal_rows_async(h, C.byref(cam), C.byref(p), 1.0, 0, hgt, 1,
                                                          d, d, None, None, None, stream.cuda_stream)
                    assert rc == 0
                e1.record(stream)
                torch.cuda.synchronize()
                if r == 0:
                    imgs[name] = outs[name].cpu().numpy()
                elif r >= 2:
                    times[name].append(e0.elapsed_time(e1) / nb)
        base = imgs["base"]
        for name in handles:
            t = np.array(times[name])
            same = bool(np.array_equal(imgs[name], base))
            res[f"{name}/{cfg}"] = dict(median_ms=float(np.median(t)), min_ms=float(t.min()),
                                        identical_to_base=same)
            print(f"{cfg} {name:>12s} median {np.median(t):.4f} ms  min {t.min():.4f} ms  "
                  f"identical={same}", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
