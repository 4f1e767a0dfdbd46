#!/usr/bin/env python3
"""Diagnostic: exact-walk work per rank of a K-way block-cyclic split (ABI v11 row blocks).

Renders the config's frame once with hit records (exact STATS instance) and sums each pixel's
DDA + shadow-DDA steps (vrt_hit.steps) per frame row, then per rank for several row-block sizes,
so that a band that rehearses slower than its peers (bench.py --rehearse-rank) can be told apart
from one that simply holds more work. Prints one JSON object.
Usage: python scripts/band_cost.py [--config C3] [--ranks 8] [--blocks 16,8,4]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraytracer_amd as vrt  # noqa: E402
from bench import CONFIGS  # noqa: E402
from voxelraytracer_amd.tiles import block_band_spec, band_frame_rows  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--blocks", default="16,8,4")
a = ap.parse_args()
scene, n, w, h, R, T, _ = CONFIGS[a.config]
vox = vrt.build_scene(scene, n)
with vrt.Renderer(0) as r:
    r.upload_volume(vox, n)
    _, hits, stats = r.render(vrt.make_camera(w, h), vrt.default_params(R, T), want_hits=True, counters=True)
steps = hits["steps"].astype(np.int64)
row = steps.sum(axis=1)
out = {"config": a.config, "ranks": a.ranks, "frame_steps": int(row.sum()),
       "row_steps_top": sorted(((int(v), i) for i, v in enumerate(row)), reverse=True)[:12],
       "pixel_steps_max": int(steps.max()), "split": {}}
for b in (int(x) for x in a.blocks.split(",")):
    per = []
    for k in range(a.ranks):
        row0, rows, step = block_band_spec(k, a.ranks, h, b)
        idx = band_frame_rows(row0, rows, step, b).numpy() if rows else np.zeros(0, dtype=np.int64)
        per.append({"rank": k, "rows": int(rows), "steps": int(row[idx].sum()),
                    "max_pixel": int(steps[idx].max()) if rows else 0})
    mean = sum(p["steps"] for p in per) / a.ranks
    out["split"][f"block{b}"] = {"max_over_mean": round(max(p["steps"] for p in per) / mean, 4), "ranks": per}
print(json.dumps(out, indent=1))
