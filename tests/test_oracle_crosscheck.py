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
    d = dict(sun_dir=list(p.sun_dir), time=p.time, ray_noise=p.ray_noise,
             reflection_noise=p.reflection_noise, refraction_noise=p.refraction_noise,
             max_ray_length=p.max_ray_length, max_reflections=p.max_reflections,
             max_transparencies=p.max_transparencies, color_only=p.color_only)
    if not p.color_only:
        d.update(atlas=p._atlas_ref, atlas_size=p.atlas_size,
                 atlas_texture_size=p.atlas_texture_size)
    return d


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


TEXTURED = [
    # textured mode (voxel.glsl without _COLOR_ONLY): atlas colours at the hit's face plane, the
    # textured material table, alpha-driven refraction push and energy
    ("terrain", 16, 20, 14, 4, 2, {}),
    ("glass_cube", 16, 18, 14, 4, 4, dict(ray_noise=0.05, reflection_noise=0.05, time=3.0)),
    ("refraction", 16, 16, 12, 4, 4, dict(pos=(0.4, -0.3, 0.2), rot=(12.0, 160.0, 0.0))),
    ("glass_cube", 16, 15, 15, 4, 4, dict(pos=(0.25, 0.25, 0.25), rot=(-35.26439, 45.0, 0.0))),
]


@pytest.mark.parametrize("case", TEXTURED, ids=[f"tex_{c[0]}{c[1]}_{i}" for i, c in enumerate(TEXTURED)])
@pytest.mark.parametrize("atlas_size,ts", [(256, 128), (32, 16)])
def test_textured_c_oracle_matches_numpy(built, case, atlas_size, ts):
    scene, n, w, h, R, T, extra = case
    extra = dict(extra)
    cam = vrt.make_camera(w, h, **{k: extra.pop(k) for k in ("pos", "rot") if k in extra})
    p = vrt.textured_params(vrt.default_params(R, T, **extra), vrt.make_atlas(atlas_size, ts), ts)
    vox = vrt.build_scene(scene, n)
    rgba_c, hits_c, cnt_c = oracle.render(cam, vox, n, p, threads=1)
    rgba_n, hits_n, cnt_n = numpy_oracle.render(list(cam.inv_pv), w, h, vox, n, params_dict(p))
    assert np.array_equal(hits_c["voxel_index"], hits_n["voxel_index"])
    assert np.array_equal(hits_c["ray_length"].view(np.uint32), hits_n["ray_length"].view(np.uint32))
    assert np.array_equal(hits_c["steps"], hits_n["steps"])
    assert cnt_c == cnt_n
    assert np.abs(np.clip(rgba_c, 0, 1) - np.clip(rgba_n, 0, 1)).max() <= 1e-5
    # textured shading really differs from colour-only on these frames
    rgba_0, _, _ = oracle.render(cam, vox, n, vrt.default_params(R, T, **extra), threads=1)
    assert np.abs(rgba_0 - rgba_c).max() > 1e-3


def test_texture_coordinate_known_answers(built):
    """GetTextureCoordinate (:167-172) + NEAREST/REPEAT fetch, hand-derived: atlas 256, tiles 128,
    point (3.25, 7.5, 1.0) on a z face (index 2 -> plane (x, y) = (3.25, 7.5), frac (0.25, 0.5))."""
    S = 256
    atlas = np.zeros((S, S, 4), np.uint8)
    atlas[..., 0] = np.arange(S, dtype=np.uint8)[None, :]    # R = column
    atlas[..., 1] = np.arange(S, dtype=np.uint8)[:, None]    # G = row
    atlas[..., 3] = 255
    pt = (3.25, 7.5, 1.0)
    # stone (0,0): u = 0.25*128/256 = 0.125 -> col 32; v = 1 - (1-0.5)*0.5 = 0.75 -> row 192
    assert list(oracle.get_color(atlas, S, 128, 1, pt, 2)[:2] * 255) == [32, 192]
    # glass (0,1): v = 1 - (0.5 + 1)*0.5 = 0.25 -> row 64
    assert list(oracle.get_color(atlas, S, 128, 2, pt, 2)[:2] * 255) == [32, 64]
    # grass (1,1): u = (0.25 + 1)*0.5 = 0.625 -> col 160
    assert list(oracle.get_color(atlas, S, 128, 3, pt, 2)[:2] * 255) == [160, 64]
    # x face (index 0): plane (z, y) = (1.0, 7.5) -> frac (0, 0.5): col 0 of the stone slot
    assert list(oracle.get_color(atlas, S, 128, 1, pt, 0)[:2] * 255) == [0, 192]
    # y face (index 1): plane (x, z) = (3.25, 1.0) -> frac (0.25, 0): v = 1 - 0.5 = 0.5 -> row 128
    assert list(oracle.get_color(atlas, S, 128, 1, pt, 1)[:2] * 255) == [32, 128]
    # colour-only mode returns the material table colour (:71-87)
    assert np.allclose(oracle.get_color(atlas, S, 128, 3, pt, 2, textured=False),
                       [0.05, 0.5, 0.1, 1.0])


def test_oracle_trace_pixel(built):
    """The oracle's per-pixel ray-tree trace (debug tooling for certified trees): the traced pixel's
    colour equals oracle.render's, and a glass pixel of the glass cube traces its primary hit, its
    refraction ray's in-volume refraction out of the wall and its reflection ray, DFS order."""
    import oracle
    import voxelraytracer_amd as vrt

    n, w, h = 16, 40, 30
    vox = vrt.build_scene("glass_cube", n)
    cam = vrt.make_camera(w, h)
    p = vrt.default_params(1, 2)
    img, _, _ = oracle.render(cam, vox, n, p)
    for px, py in ((3, 4), (20, 15), (37, 27)):
        recs, rgba = oracle.trace_pixel(cam, vox, n, p, px, py)
        assert np.array_equal(rgba.view(np.uint32), img[py, px].view(np.uint32))
        calls = recs[recs[:, 0] == 1]
        assert calls[0, 1] == 1 and calls[0, 2] == 2          # the primary hits glass
        assert calls[1, 17] == 2 and calls[1, 19] == 1        # popped first: the refraction ray
        assert (recs[:, 0] == 10).any()                       # it leaves the wall by in-volume refraction
        assert calls[2, 18] == 1                               # then the reflection ray
