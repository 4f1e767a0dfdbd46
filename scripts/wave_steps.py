#!/usr/bin/env python3
"""Per-wave exact step totals of a BASELINE config (analysis only): renders with hit records
(exact walks, per-pixel steps) and prints the waves (8x8 pixel tiles) with the largest max / sum
of steps, next to the wave timeline of scripts/stamps.py when its npz is given.
Usage: python scripts/wave_steps.py [--config C3] [--stamps gpurun_out/x/stamps_C3.npz]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import voxelraytracer_amd as vrt  # noqa: E402
from bench import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--stamps", default="")
a = ap.parse_args()
scene, n, w, h, R, T, desc = CONFIGS[a.config]
r = vrt.Renderer(0)
r.upload_volume(vrt.build_scene(scene, n), n)
cam = vrt.make_camera(w, h)
p = vrt.default_params(R, T)
_, hits, st = r.render(cam, p)
steps = hits["steps"].astype(np.int64)
flags = hits["flags"]
H8, W8 = (h + 7) // 8, (w + 7) // 8
pad = np.zeros((H8 * 8, W8 * 8), np.int64)
pad[:h, :w] = steps
tiles = pad.reshape(H8, 8, W8, 8).transpose(0, 2, 1, 3).reshape(H8, W8, 64)
tmax, tsum = tiles.max(-1), tiles.sum(-1)
print(f"{a.config}: pixel steps mean {steps.mean():.1f} p99 {np.percentile(steps, 99):.0f} max {steps.max()}")
print(f"wave max-steps quantiles p50 {np.percentile(tmax, 50):.0f} p90 {np.percentile(tmax, 90):.0f} "
      f"p99 {np.percentile(tmax, 99):.0f} max {tmax.max()}")
order = np.argsort(-tmax.reshape(-1))[:15]
dur = None
if a.stamps:
    d = np.load(a.stamps)["stamps"].astype(np.int64)
    gx = (w + 15) // 16
    t0 = d[:, 0].min()
    du = (d[:, 1] - d[:, 0]) / 100.0
    d2 = np.load(a.stamps)["stamps2"].astype(np.int64) if "stamps2" in np.load(a.stamps).files else None
    dur = np.zeros((H8, W8))
    cpart = np.zeros((H8, W8))
    nex = np.zeros((H8, W8), np.int64)
    for i in range(len(d)):
        blk, wv = divmod(i, 4)
        ty, tx = (blk // gx) * 2 + (wv >> 1), (blk % gx) * 2 + (wv & 1)
        if ty < H8 and tx < W8:
            dur[ty, tx] = du[i]
            if d2 is not None:
                cpart[ty, tx] = (d2[i, 0] - d[i, 0]) / 100.0
                nex[ty, tx] = d2[i, 1]
    print(f"corr(wave max steps, duration) {np.corrcoef(tmax.ravel(), dur.ravel())[0,1]:.3f}; "
          f"corr(sum steps, duration) {np.corrcoef(tsum.ravel(), dur.ravel())[0,1]:.3f}")
for i in order:
    ty, tx = divmod(int(i), W8)
    px = tiles[ty, tx]
    j = int(np.argmax(px))
    extra = f" dur {dur[ty, tx]:.1f} us" if dur is not None else ""
    print(f"wave tile ({tx},{ty}) px ({tx*8 + j % 8},{ty*8 + j // 8}) max {tmax[ty, tx]} sum {tsum[ty, tx]}"
          f" flags {flags[min(ty*8 + j // 8, h - 1), min(tx*8 + j % 8, w - 1)]:#x}{extra}")
if dur is not None:
    o = np.argsort(-dur.ravel())[:25]
    print("longest waves by duration:")
    for i in o:
        ty, tx = divmod(int(i), W8)
        print(f"  tile ({tx},{ty}) dur {dur[ty, tx]:.1f} us (certified part {cpart[ty, tx]:.1f} us, "
              f"exact lanes {nex[ty, tx]})  max steps {tmax[ty, tx]} sum {tsum[ty, tx]}")
r.close()
