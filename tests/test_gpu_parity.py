"""GPU parity: the gfx950 HIP kernel (through the C-ABI) against the CPU oracle.

Contract (DESIGN.md "Numerics"):
  - hit records bit-exact: primary-hit voxel index, ray length bits, per-pixel step count, flags
  - counters (rays, DDA steps, probes, ties) exact
  - colour: |clamp(rgb,0,1)_gpu - clamp(rgb,0,1)_oracle| <= 1e-4 (COLOR_TOL); pow() goes through
    exp2/log2, whose last-ulp behaviour differs between the GPU and glibc
"""
import os

import numpy as np
import pytest

import oracle
import voxelraytracer_amd as vrt

pytestmark = pytest.mark.gpu

COLOR_TOL = 1e-4
THREADS = min(16, os.cpu_count() or 1)   # the GPU box's CPU share


@pytest.fixture(scope="module")
def renderer(built):
    r = vrt.Renderer(0)
    yield r
    r.close()


def compare(rgba_g, hits_g, cnt_g, rgba_o, hits_o, cnt_o):
    assert np.array_equal(hits_g["voxel_index"], hits_o["voxel_index"])
    assert np.array_equal(hits_g["ray_length"].view(np.uint32), hits_o["ray_length"].view(np.uint32))
    assert np.array_equal(hits_g["steps"], hits_o["steps"])
    assert np.array_equal(hits_g["flags"], hits_o["flags"])
    for k in oracle.COUNTER_NAMES:
        assert cnt_g[k] == cnt_o[k], k
    d = np.abs(np.clip(rgba_g[..., :3], 0, 1) - np.clip(rgba_o[..., :3], 0, 1))
    assert d.max() <= COLOR_TOL, float(d.max())
    assert np.all(rgba_g[..., 3] == 1.0)


def run_both(renderer, scene, n, w, h, refl, transp, **kw):
    vox = vrt.build_scene(scene, n)
    renderer.upload_volume(vox, n)
    cam = vrt.make_camera(w, h, **{k: kw.pop(k) for k in ("pos", "rot") if k in kw})
    p = vrt.default_params(refl, transp, **kw)
    rgba_g, hits_g, st = renderer.render(cam, p)
    rgba_o, hits_o, cnt_o = oracle.render(cam, vox, n, p, threads=THREADS)
    return (rgba_g, hits_g, st), (rgba_o, hits_o, cnt_o)


CASES = [
    # (scene, N, W, H, R, T, extra)  -- C0 is BASELINE.json configs[0] verbatim
    ("glass_cube", 16, 400, 400, 1, 2, {}),
    ("glass_cube", 16, 128, 128, 1, 2, dict(ray_noise=0.05, reflection_noise=0.05,
                                            refraction_noise=0.01, time=7.0)),
    ("glass_cube", 32, 96, 64, 4, 4, {}),
    ("terrain", 16, 128, 128, 4, 2, {}),
    ("terrain", 32, 160, 90, 4, 2, dict(ray_noise=0.02, time=3.0)),
    ("terrain", 64, 160, 90, 4, 4, {}),
    ("refraction", 32, 128, 72, 4, 4, {}),
    ("refraction", 16, 100, 60, 0, 0, {}),
    ("terrain", 128, 256, 144, 4, 2, {}),
    ("refraction", 128, 192, 108, 4, 4, dict(pos=(0.3, -0.2, 0.1), rot=(10.0, 170.0, 0.0))),
    ("glass_cube", 64, 96, 96, 8, 8, dict(pos=(1.0, 2.0, -3.0), rot=(-60.0, 20.0, 0.0))),
    # degenerate geometry: +0 direction components (exact fallback walk), a -6e-17 component
    # (Markstein division with ~1e16 reciprocals), zero-t ties incl. the index-3 (y+z) tie
    ("glass_cube", 16, 9, 9, 4, 4, dict(pos=(0.0, 0.0, 0.0), rot=(0.0, 0.0, 0.0))),
    ("glass_cube", 128, 65, 65, 4, 4, dict(pos=(0.0, 0.0, 0.0), rot=(0.0, 0.0, 0.0))),
    ("refraction", 16, 9, 7, 4, 4, dict(pos=(0.0, 0.0, 0.0), rot=(0.0, 90.0, 0.0))),
    ("glass_cube", 16, 15, 15, 4, 4, dict(pos=(0.25, 0.25, 0.25), rot=(-35.26439, 45.0, 0.0))),
    ("terrain", 32, 121, 121, 4, 2, dict(pos=(0.0, 5.0, 0.0), rot=(-90.0, 0.0, 0.0))),
    ("terrain", 512, 384, 216, 4, 2, {}),
    # deep bounce trees (the largest stack the ABI accepts, R + T + 1 = 17): the stack order of
    # reflection rays parked under refraction rays, tdepth-heavy and rdepth-heavy
    ("glass_cube", 32, 128, 96, 4, 12, dict(pos=(0.5, 1.0, -2.5), rot=(-25.0, 15.0, 0.0))),
    ("refraction", 64, 128, 72, 12, 4, dict(ray_noise=0.02, refraction_noise=0.02, time=5.0)),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}{c[1]}_{c[2]}x{c[3]}_R{c[4]}T{c[5]}_{i}"
                                             for i, c in enumerate(CASES)])
def test_parity_small(renderer, case):
    scene, n, w, h, R, T, extra = case
    (rg, hg, st), (ro, ho, co) = run_both(renderer, scene, n, w, h, R, T, **dict(extra))
    compare(rg, hg, st, ro, ho, co)


@pytest.mark.parametrize("scene,R,T", [("glass_cube", 1, 2), ("terrain", 4, 2), ("refraction", 4, 4)])
def test_parity_full_size_baseline_configs(renderer, scene, R, T):
    """BASELINE.json configs[1..3]: 1920x1080 at 128^3, the whole frame against the oracle."""
    (rg, hg, st), (ro, ho, co) = run_both(renderer, scene, 128, 1920, 1080, R, T)
    compare(rg, hg, st, ro, ho, co)


def test_parity_full_size_c4(renderer):
    """BASELINE.json configs[4] at full size: _TERRAIN 512^3, 3840x2160, (R,T)=(4,2)."""
    (rg, hg, st), (ro, ho, co) = run_both(renderer, "terrain", 512, 3840, 2160, 4, 2)
    compare(rg, hg, st, ro, ho, co)


def test_row_bands_compose_to_full_frame(renderer):
    """Cyclic and contiguous row bands (the multi-GPU tiling) reproduce the full frame exactly."""
    import torch

    n, w, h = 32, 96, 60
    vox = vrt.build_scene("terrain", n)
    renderer.upload_volume(vox, n)
    cam = vrt.make_camera(w, h)
    p = vrt.default_params(4, 2)
    full, fhits, _ = renderer.render(cam, p)
    for k in (2, 3, 4):
        rows = h // k
        out = torch.empty((k, rows, w, 4), dtype=torch.float32, device="cuda")
        cnt = torch.zeros((k, len(oracle.COUNTER_NAMES)), dtype=torch.int64, device="cuda")
        for r in range(k):   # cyclic: rank r owns frame rows r, r+k, ...
            renderer.render_rows_async(cam, p, r, rows, k, out[r].data_ptr(), 0, cnt[r].data_ptr())
        torch.cuda.synchronize()
        frame = out.permute(1, 0, 2, 3).reshape(h, w, 4).cpu().numpy()
        assert np.array_equal(frame, full)
        for r in range(k):   # contiguous bands
            renderer.render_rows_async(cam, p, r * rows, rows, 1, out[r].data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(out.reshape(h, w, 4).cpu().numpy(), full)


TEXTURED = [
    # textured mode (voxel.glsl without _COLOR_ONLY): (scene, N, W, H, R, T, atlas, tile, extra)
    ("terrain", 16, 128, 96, 4, 2, 256, 128, {}),
    ("terrain", 64, 160, 90, 4, 4, 32, 16, dict(ray_noise=0.02, time=3.0)),
    ("glass_cube", 32, 128, 96, 4, 4, 256, 128, dict(reflection_noise=0.05, time=2.0)),
    ("refraction", 128, 192, 108, 4, 4, 256, 128, {}),
    ("glass_cube", 16, 15, 15, 4, 4, 256, 128, dict(pos=(0.25, 0.25, 0.25),
                                                    rot=(-35.26439, 45.0, 0.0))),
]


@pytest.mark.parametrize("case", TEXTURED, ids=[f"tex_{c[0]}{c[1]}_{c[6]}_{i}"
                                                for i, c in enumerate(TEXTURED)])
def test_parity_textured(renderer, case):
    scene, n, w, h, R, T, size, ts, extra = case
    extra = dict(extra)
    vox = vrt.build_scene(scene, n)
    renderer.upload_volume(vox, n)
    cam = vrt.make_camera(w, h, **{k: extra.pop(k) for k in ("pos", "rot") if k in extra})
    p = vrt.textured_params(vrt.default_params(R, T, **extra), vrt.make_atlas(size, ts), ts)
    rgba_g, hits_g, st = renderer.render(cam, p)
    rgba_o, hits_o, cnt_o = oracle.render(cam, vox, n, p, threads=THREADS)
    compare(rgba_g, hits_g, st, rgba_o, hits_o, cnt_o)


def test_parity_textured_full_size_refraction(renderer):
    """C3's frame (1920x1080, 128^3, (4,4)) in textured mode, the reference's default build."""
    vox = vrt.build_scene("refraction", 128)
    renderer.upload_volume(vox, 128)
    cam = vrt.make_camera(1920, 1080)
    p = vrt.textured_params(vrt.default_params(4, 4), vrt.make_atlas())
    rgba_g, hits_g, st = renderer.render(cam, p)
    rgba_o, hits_o, cnt_o = oracle.render(cam, vox, 128, p, threads=THREADS)
    compare(rgba_g, hits_g, st, rgba_o, hits_o, cnt_o)


def ref_atlas():
    """The reference's own textures (res/textures/*128.png, main.cpp:187-193) decoded into the
    ABI atlas layout: tests/golden/atlas/atlas_ref128.npz (tests/golden/make_atlas_ref.py)."""
    path = os.path.join(os.path.dirname(__file__), "golden", "atlas", "atlas_ref128.npz")
    return np.load(path, allow_pickle=False)["atlas"]


@pytest.mark.parametrize("scene,R,T", [("refraction", 4, 4), ("glass_cube", 1, 2)])
def test_parity_textured_full_size_reference_atlas(renderer, scene, R, T):
    """Full 1920x1080 frames at 128^3 in textured mode with the reference's own atlas, whose glass
    alpha is 0 or 255: both sides of GetColor(hit).a != 1 (voxel.glsl:445) and of
    energy *= 1 - a (:239-240) occur."""
    vox = vrt.build_scene(scene, 128)
    renderer.upload_volume(vox, 128)
    cam = vrt.make_camera(1920, 1080)
    p = vrt.textured_params(vrt.default_params(R, T), ref_atlas())
    rgba_g, hits_g, st = renderer.render(cam, p)
    rgba_o, hits_o, cnt_o = oracle.render(cam, vox, 128, p, threads=THREADS)
    compare(rgba_g, hits_g, st, rgba_o, hits_o, cnt_o)
    assert cnt_o["secondary_rays"] > 0


def test_atlas_upload_and_switching(renderer):
    """The context keeps the atlas: an explicit upload serves a params block without a pointer;
    a different pointer re-uploads; colour-only renders are unaffected."""
    vox = vrt.build_scene("terrain", 16)
    renderer.upload_volume(vox, 16)
    cam = vrt.make_camera(64, 48)
    a1, a2 = vrt.make_atlas(seed=1), vrt.make_atlas(seed=2)
    p1 = vrt.textured_params(vrt.default_params(4, 2), a1)
    ref1, _, _ = oracle.render(cam, vox, 16, p1, threads=THREADS)
    renderer.upload_atlas(a1)
    p_noptr = vrt.default_params(4, 2)
    p_noptr.color_only, p_noptr.atlas_size, p_noptr.atlas_texture_size = 0, 256, 128
    g1, _, _ = renderer.render(cam, p_noptr)
    assert np.abs(np.clip(g1, 0, 1) - np.clip(ref1, 0, 1)).max() <= COLOR_TOL
    p2 = vrt.textured_params(vrt.default_params(4, 2), a2)
    g2, _, _ = renderer.render(cam, p2)
    ref2, _, _ = oracle.render(cam, vox, 16, p2, threads=THREADS)
    assert np.abs(np.clip(g2, 0, 1) - np.clip(ref2, 0, 1)).max() <= COLOR_TOL
    assert np.abs(ref1 - ref2).max() > 1e-3
    g0, _, _ = renderer.render(cam, vrt.default_params(4, 2))
    r0, _, _ = oracle.render(cam, vox, 16, vrt.default_params(4, 2), threads=THREADS)
    assert np.abs(np.clip(g0, 0, 1) - np.clip(r0, 0, 1)).max() <= COLOR_TOL
    # the same host buffer with new bytes is re-uploaded (content, not pointer identity)
    buf = a1.copy()
    p3 = vrt.textured_params(vrt.default_params(4, 2), buf)
    renderer.render(cam, p3)
    buf[...] = a2
    g3, _, _ = renderer.render(cam, p3)
    assert np.abs(np.clip(g3, 0, 1) - np.clip(ref2, 0, 1)).max() <= COLOR_TOL


def test_errors_are_reported(renderer):
    cam = vrt.make_camera(8, 8)
    p = vrt.default_params()
    p.color_only = 0          # textured, but no atlas uploaded and none given
    p.atlas_size, p.atlas_texture_size = 64, 32
    fresh = vrt.Renderer(0)
    fresh.upload_volume(vrt.build_scene("glass_cube", 16), 16)
    with pytest.raises(vrt.VrtError) as e:
        fresh.render(cam, p)
    assert e.value.code == -1
    fresh.close()
    with pytest.raises(vrt.VrtError):
        renderer.upload_atlas(np.zeros((48, 48, 4), np.uint8))   # not a power of two
    with pytest.raises(vrt.VrtError):
        renderer.upload_volume(np.zeros(27, np.uint8), 3)   # N must be a power of two


def test_randomize_direction_bit_exact(renderer):
    """The kernel's RandomizeDirection (vrt_debug_randomize) against the oracle, bit for bit:
    random directions, directions with exact +0 / -0 components (where the hash decides the sign
    of a zero at noise 0, voxel.glsl:132-140), at noise +0, -0 and > 0."""
    rng = np.random.default_rng(11)
    n = 512
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    z = np.float32(0.0)
    nz = np.float32(-0.0)
    d[0:64, 0] = nz
    d[64:128, 1] = nz
    d[128:192, 2] = z
    d[192:256, 0] = nz
    d[192:256, 2] = nz
    d[256:272] = [z, nz, np.float32(1.0)]
    p = (rng.uniform(-2, 130, size=(n, 3))).astype(np.float32)
    for randomness, seed in [(0.0, 1.0), (-0.0, 3.0), (0.05, 7.0), (1.0, 2.0)]:
        got = renderer.debug_randomize(d, p, randomness, seed)
        ref = np.stack([oracle.randomize_direction(d[i], p[i], randomness, seed) for i in range(n)])
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), randomness
    # at noise 0 the -0 components really do depend on the hash (both signs occur)
    got = renderer.debug_randomize(d[:64], p[:64], 0.0, 1.0)
    signs = np.signbit(got[:, 0])
    assert signs.any() and (~signs).any()


@pytest.mark.parametrize("scene,n,R,T", [("refraction", 128, 4, 4), ("glass_cube", 128, 1, 2),
                                         ("terrain", 128, 4, 2), ("terrain", 32, 4, 2)])
def test_textured_fast_path_equals_exact_instance(renderer, scene, n, R, T):
    """Stats-free textured frames (exact walks with certified shadow walks from the exact hit
    points, CERT 1) equal the exact instance's bit for bit, with the reference atlas, at full
    size; terrain 32^3 has glass walls (main.cpp:233)."""
    vox = vrt.build_scene(scene, n)
    renderer.upload_volume(vox, n)
    cam = vrt.make_camera(1920, 1080)
    p = vrt.textured_params(vrt.default_params(R, T), ref_atlas())
    exact, _, _ = renderer.render(cam, p, want_hits=False, counters=True)
    fast, _, st = renderer.render(cam, p, want_hits=False, counters=False)
    assert st["kernel_ms"] > 0
    assert np.array_equal(fast.view(np.uint32), exact.view(np.uint32))
