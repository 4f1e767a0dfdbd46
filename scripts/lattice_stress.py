#!/usr/bin/env python3
"""Stress: certified frames (trees on / off, deferred exact pass and in lane) against the exact STATS
instance on lattice-aligned cameras — integer and half-integer positions, axis-aligned, diagonal and
(1,1,1) views — over glass-heavy and glass-light scenes; prints every mismatching case. Usage:
python scripts/lattice_stress.py [cameras per scene] [scene:n,...]"""
import itertools
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraytracer_amd as vrt  # noqa: E402


def frame(r, cam, p, counters=False):
    h, w = cam.height, cam.width
    buf = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(len(vrt.COUNTER_NAMES), dtype=torch.int64, device="cuda")
    r.render_temporal_rows_async(cam, p, 1.0, 0, h, 1, buf.data_ptr(), buf.data_ptr(),
                                 d_counters=cnt.data_ptr() if counters else 0,
                                 stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return buf.cpu().numpy()


def main():
    per = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    rng = np.random.default_rng(7)
    pitches = [0.0, -45.0, 45.0, -35.26439, -90.0, 90.0, -30.0, -60.0, -89.99]
    yaws = [0.0, 45.0, 90.0, 135.0, 180.0, 225.0, 270.0, 315.0, 30.0, 60.0]
    scenes = [("glass_cube", 64), ("glass_cube", 128), ("refraction", 64), ("refraction", 128), ("terrain", 64),
              ("terrain", 128)]
    if len(sys.argv) > 2:
        scenes = [(s_.split(":")[0], int(s_.split(":")[1])) for s_ in sys.argv[2].split(",")]
    total = bad_cases = 0
    with vrt.Renderer(0) as r:
        r.set_certified(1)
        for scene, n in scenes:
            r.upload_volume(vrt.build_scene(scene, n), n)
            for k in range(per):
                pos = tuple(float(x) for x in np.round(rng.uniform(-n / 2.5, n / 2.5, 3) * 2) / 2)
                if k % 3 == 0:
                    pos = tuple(float(round(x)) for x in pos)
                rot = (float(rng.choice(pitches)), float(rng.choice(yaws)), 0.0)
                R, T = [(4, 4), (1, 2), (2, 6)][k % 3]
                cam = vrt.make_camera(320, 180, pos=pos, rot=rot)
                p = vrt.default_params(R, T, time=1.0)
                ref = frame(r, cam, p, counters=True)
                for trees, ep in itertools.product((2, 0), (2, 0)):
                    r.set_cert_trees(trees)
                    r.set_exact_pass(ep)
                    got = frame(r, cam, p)
                    total += 1
                    bad = np.argwhere(np.any(got != ref, axis=-1))
                    if bad.size:
                        bad_cases += 1
                        y, x = bad[0]
                        print(f"MISMATCH {scene}{n} pos={pos} rot={rot} RT=({R},{T}) trees={trees} ep={ep}: "
                              f"{len(bad)} px, first ({x},{y}) got {got[y, x].tolist()} ref {ref[y, x].tolist()}",
                              flush=True)
            print(f"{scene}{n}: done, {bad_cases} mismatching cases so far of {total}", flush=True)
    print(f"TOTAL {bad_cases} mismatching of {total}")


if __name__ == "__main__":
    main()
