"""Cross-check of the two independent restatements of voxel.glsl: the C oracle
(oracle/vrt_oracle.c) against the NumPy float32 one (oracle/numpy_oracle.py), on small frames.
Bit-exact on hit records and counters; colour within 1e-5 (only exp2/log2 differ: glibc vs
NumPy)."""
import numpy as np
import pytest

import oracle
import voxelraytracer_amd as vrt
from oracle import numpy_oracle

CASES = [
    # scene, N, W, H, R, T, extra params
    ("glass_cube", 16, 20, 14, 1, 2, {}),
    ("glass_cube", 16, 16, 12, 1, 2, dict(ray_noise=0.05, reflection_noise=0.05,
                                          refraction_noise=0.01, time=7.0)),
    ("terrain", 16, 18, 12, 4, 2, {}),
    ("refraction", 16, 16, 10, 4, 4, dict(pos=(0.4, -0.3, 0.2), rot=(12.0, 160.0, 0.0))),
    ("glass_cube", 8, 14, 14, 4, 4, dict(pos=(0.5, 0.25, -1.0), rot=(-50.0, 30.0, 0.0))),
    # degenerate geometry: exact +0 direction components (centre pixel, odd W/H), a -6e-17
    # component, and zero-t ties including the y+z tie that reads intersectionAxis[3]
    ("glass_cube", 16, 9, 9, 4, 4, dict(pos=(0.0, 0.0, 0.0), rot=(0.0, 0.0, 0.0))),
    ("refraction", 16, 9, 7, 4, 4, dict(pos=(0.0, 0.0, 0.0), rot=(0.0, 90.0, 0.0))),
    ("glass_cube", 16, 15, 15, 4, 4, dict(pos=(0.25, 0.25, 0.25), rot=(-35.26439, 45.0, 0.0))),
    ("glass_cube", 16, 48, 32, 1, 2, {}),
]


def params_dict(p):
    return dict(sun_dir=list(p.sun_dir), time=p.time, ray_noise=p.ray_noise,
                reflection_noise=p.reflection_noise, refraction_noise=p.refraction_noise,
                max_ray_length=p.max_ray_length, max_reflections=p.max_reflections,
                max_transparencies=p.max_transparencies)


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}{c[1]}_{i}" for i, c in enumerate(CASES)])
def test_c_oracle_matches_numpy_restatement(built, case):
    scene, n, w, h, R, T, extra = case
    extra = dict(extra)
    cam = vrt.make_camera(w, h, **{k: extra.pop(k) for k in ("pos", "rot") if k in extra})
    p = vrt.default_params(R, T, **extra)
    vox = vrt.build_scene(scene, n)
    rgba_c, hits_c, cnt_c = oracle.render(cam, vox, n, p, threads=1)
    rgba_n, hits_n, cnt_n = numpy_oracle.render(list(cam.inv_pv), w, h, vox, n, params_dict(p))
    assert np.array_equal(hits_c["voxel_index"], hits_n["voxel_index"])
    assert np.array_equal(hits_c["ray_length"].view(np.uint32), hits_n["ray_length"].view(np.uint32))
    assert np.array_equal(hits_c["steps"], hits_n["steps"])
    assert np.array_equal(hits_c["flags"], hits_n["flags"])
    assert cnt_c == cnt_n
    assert np.abs(np.clip(rgba_c, 0, 1) - np.clip(rgba_n, 0, 1)).max() <= 1e-5
