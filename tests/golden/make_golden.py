#!/usr/bin/env python3
"""Generate tests/golden/*.npz — small fixtures of the voxel.glsl hot path.

Produced by the CPU oracle (oracle/vrt_oracle.c), itself cross-checked bit-exactly against the
independent NumPy restatement (tests/test_oracle_crosscheck.py). The reference ships no golden
vectors and cannot run here, so these pin REGRESSIONS of the restatement and the
kernel, not the reference's own output. Each fixture holds its inputs (scene id, N, seed, camera
matrix, params) and outputs (RGBA float32, primary hit records, counters) plus the SHA-256 of the
volume bytes, which pins the scene builders (main.cpp:218-288).
Usage: python tests/golden/make_golden.py [fixture names]
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
import voxelraytracer_amd as vrt  # noqa: E402

FIXTURES = [
    # name, scene, N, W, H, R, T, extra params
    ("c0_glass_cube16_64", "glass_cube", 16, 64, 64, 1, 2, {}),
    ("glass_cube16_noise_64", "glass_cube", 16, 64, 64, 1, 2,
     dict(ray_noise=0.05, reflection_noise=0.05, refraction_noise=0.01, time=7.0)),
    ("terrain16_64", "terrain", 16, 64, 64, 4, 2, {}),
    ("terrain32_glass_walls_96x54", "terrain", 32, 96, 54, 4, 2, {}),
    ("refraction16_64", "refraction", 16, 64, 64, 4, 4, {}),
    ("glass_cube16_axis_aligned_33", "glass_cube", 16, 33, 33, 4, 4,
     dict(pos=(0.0, 0.0, 0.0), rot=(0.0, 0.0, 0.0))),
    # textured mode (the reference's default build); the fixture stores its 32x32 atlas
    ("textured_terrain16_64", "terrain", 16, 64, 64, 4, 2, dict(atlas=(32, 16, 5))),
    ("textured_glass_cube16_48", "glass_cube", 16, 48, 48, 4, 4,
     dict(atlas=(32, 16, 6), reflection_noise=0.05, time=2.0)),
    # textured mode with the reference's own textures (tests/golden/atlas/atlas_ref128.npz, made
    # by make_atlas_ref.py from res/textures/*128.png): glass alpha is 0 or 255, so both sides of
    # GetColor(hit).a != 1 (voxel.glsl:445) and energy *= 1 - a (:239-240) occur
    ("textured_ref_refraction32_96x64", "refraction", 32, 96, 64, 4, 4, dict(atlas="ref")),
    ("textured_ref_glass_cube16_64", "glass_cube", 16, 64, 64, 4, 4,
     dict(atlas="ref", reflection_noise=0.05, time=2.0)),
]


def ref_atlas():
    z = np.load(os.path.join(HERE, "atlas", "atlas_ref128.npz"), allow_pickle=False)
    return z["atlas"]

PARAM_KEYS = ("time", "ray_noise", "reflection_noise", "refraction_noise", "max_ray_length",
              "max_reflections", "max_transparencies", "color_only", "atlas_size",
              "atlas_texture_size")


def main(only=()):
    for name, scene, n, w, h, R, T, extra in FIXTURES:
        if only and name not in only:
            continue
        extra = dict(extra)
        pose = {k: extra.pop(k) for k in ("pos", "rot") if k in extra}
        cam = vrt.make_camera(w, h, **pose)
        atlas_spec = extra.pop("atlas", None)
        p = vrt.default_params(R, T, **extra)
        atlas = np.zeros((0, 0, 4), np.uint8)
        if atlas_spec == "ref":
            atlas, ts = ref_atlas(), 128
            p = vrt.textured_params(p, atlas, ts)
        elif atlas_spec:
            size, ts, seed = atlas_spec
            atlas = vrt.make_atlas(size, ts, seed)
            p = vrt.textured_params(p, atlas, ts)
        vox = vrt.build_scene(scene, n)
        rgba, hits, cnt = oracle.render(cam, vox, n, p, threads=8)
        params = {k: getattr(p, k) for k in PARAM_KEYS}
        params["sun_dir"] = list(p.sun_dir)
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"),
            meta=np.array(json.dumps(dict(scene=scene, n=n, seed=0, width=w, height=h,
                                          params=params, pose=pose, counters=cnt,
                                          volume_sha256=hashlib.sha256(vox.tobytes()).hexdigest()))),
            inv_pv=np.array(cam.inv_pv, np.float32),
            rgba=rgba,
            voxel_index=hits["voxel_index"],
            ray_length_bits=hits["ray_length"].view(np.uint32),
            steps=hits["steps"],
            flags=hits["flags"],
            atlas=atlas,
        )
        print(name, cnt)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))   # optional fixture names: regenerate only those
