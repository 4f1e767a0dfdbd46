"""GPU: the deferred exact pass (vrt_set_exact_pass, ABI v9). A certified pass renders the pixels
its certified walks settle and appends the others to a list (per wave a ballot of the deferred
lanes, one atomicAdd on one of 8 XCD-local segment counters, mbcnt ranks; waves with >= 32
deferred pixels keep an 8x8 chunk in lane order); a second kernel renders the list with the exact
path, a chunk or a batch of list entries to a wave (these band sizes are under four dispatch rounds:
the short-band instance with 16-pixel sparse batches; whole frames, 64-pixel batches at 7 waves, are
checked frame by frame in test_gpu_bench_path.py). Images must be bit-identical
to the in-lane fallback and to the exact STATS instance, frame after frame, on scenes where many
pixels defer (glass cube: most pixels; random sparse volumes with every byte; near-edge cameras)
and with the temporal filter reading its history (alpha 0.5), including bands (row steps),
pitched output and band heights that leave partial tiles."""
import numpy as np
import pytest
import torch

import voxelraytracer_amd as vrt

pytestmark = pytest.mark.gpu


def frames(r, cam, n_frames, R, T, alpha, row0, rows, step, w, exact_pass, counters=False, **kw):
    r.set_exact_pass(exact_pass)
    hist = torch.zeros((rows, w, 4), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(len(vrt.COUNTER_NAMES), dtype=torch.int64, device="cuda")
    out = []
    for t in range(n_frames):
        p = vrt.default_params(R, T, time=float(t + 1), **kw)
        r.render_temporal_rows_async(cam, p, alpha, row0, rows, step, hist.data_ptr(), hist.data_ptr(),
                                     d_counters=cnt.data_ptr() if counters else 0,
                                     stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        out.append(hist.cpu().numpy().copy())
    return out


def random_volume(n, seed, density=0.02):
    rng = np.random.default_rng(seed)
    v = np.zeros(n ** 3, np.uint8)
    idx = rng.choice(n ** 3, int(density * n ** 3), replace=False)
    v[idx] = rng.integers(1, 6, len(idx))
    return v


CASES = [
    ("refraction", 128, 480, 270, 4, 4, 0, 270, 1, {}),
    ("glass_cube", 64, 320, 180, 1, 2, 0, 180, 1, {}),
    ("terrain", 128, 384, 216, 4, 2, 1, 53, 4, dict(ray_noise=0.02)),
    ("random", 32, 256, 150, 4, 4, 0, 150, 1, {}),
    ("random", 64, 200, 99, 2, 3, 2, 33, 3, dict(reflection_noise=0.01)),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}{c[1]}_{c[2]}x{c[3]}" for c in CASES])
def test_exact_pass_is_bit_identical(built, case):
    scene, n, w, h, R, T, row0, rows, step, kw = case
    vox = random_volume(n, n) if scene == "random" else vrt.build_scene(scene, n)
    with vrt.Renderer(0) as r:
        r.upload_volume(vox, n)
        r.set_certified(1)   # certified pixels also on glass-heavy volumes: many deferred pixels
        cam = vrt.make_camera(w, h)
        a = frames(r, cam, 3, R, T, 0.5, row0, rows, step, w, 2, **kw)   # deferred, any size
        b = frames(r, cam, 3, R, T, 0.5, row0, rows, step, w, 0, **kw)
        ref = frames(r, cam, 3, R, T, 0.5, row0, rows, step, w, 2, counters=True, **kw)
    for k in range(3):
        assert np.array_equal(a[k], ref[k]), f"exact pass, frame {k}"
        assert np.array_equal(b[k], ref[k]), f"in-lane, frame {k}"


def test_exact_pass_lattice_cameras(built):
    """Cameras on lattice points and diagonals (exact ties: many near-edge, deferred pixels)."""
    n, w, h = 64, 160, 90
    vox = vrt.build_scene("refraction", n)
    with vrt.Renderer(0) as r:
        r.upload_volume(vox, n)
        for pos, rot in [((0.0, 0.0, 0.0), (-45.0, -45.0, 0.0)), ((1.0, 2.0, -3.0), (0.0, 0.0, 0.0)),
                         ((-2.5, 0.5, 1.5), (-35.26439, 45.0, 0.0))]:
            cam = vrt.make_camera(w, h, pos=pos, rot=rot)
            a = frames(r, cam, 1, 4, 4, 1.0, 0, h, 1, w, 2)
            ref = frames(r, cam, 1, 4, 4, 1.0, 0, h, 1, w, 2, counters=True)
            assert np.array_equal(a[0], ref[0]), pos


def test_exact_pass_toggled_between_frames(built):
    """The exact pass switched on and off between frames on one stream: the deferred-pixel list's
    counter sets are reset whenever the slot's previous launch was not a deferred one."""
    n, w, h = 128, 320, 180
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene("refraction", n), n)
        cam = vrt.make_camera(w, h)
        hist = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda")
        ref = torch.zeros_like(hist)
        cnt = torch.zeros(len(vrt.COUNTER_NAMES), dtype=torch.int64, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        for t, on in enumerate([2, 0, 2, 2, 0, 0, 2, 1, 2]):
            p = vrt.default_params(4, 4, time=float(t + 1), ray_noise=0.01 * (t % 2))
            r.set_exact_pass(on)
            r.render_temporal_rows_async(cam, p, 0.5, 0, h, 1, hist.data_ptr(), hist.data_ptr(), stream=s)
            r.render_temporal_rows_async(cam, p, 0.5, 0, h, 1, ref.data_ptr(), ref.data_ptr(),
                                         d_counters=cnt.data_ptr(), stream=s)
            torch.cuda.synchronize()
            assert torch.equal(hist, ref), f"frame {t} (exact pass {on})"


def ref_atlas():
    """The reference's own textures (res/textures/*128.png) in the ABI atlas layout."""
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "atlas", "atlas_ref128.npz")
    return np.load(path, allow_pickle=False)["atlas"]


TEX_CASES = [
    ("refraction", 128, 480, 270, 4, 4, "ref"),
    ("terrain", 128, 384, 216, 4, 2, "ref"),
    ("glass_cube", 64, 320, 180, 1, 2, "synthetic"),
    ("refraction", 64, 256, 144, 2, 2, "synthetic"),
]


@pytest.mark.parametrize("case", TEX_CASES, ids=[f"{c[0]}{c[1]}_{c[6]}" for c in TEX_CASES])
def test_textured_certified_pixels_bit_identical(built, case):
    """Textured frames (the reference's default build, voxel.glsl:6) with certified pixels: the
    texel of a certified hit is certified from the hit's error interval on its face plane
    (cert_texel), the rest is deferred to the exact pass. Identical to the exact instance and to
    the in-lane path (exact primaries), frame after frame at alpha 0.5."""
    scene, n, w, h, R, T, which = case
    atlas = ref_atlas() if which == "ref" else vrt.make_atlas()
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene(scene, n), n)
        r.set_certified(1)
        cam = vrt.make_camera(w, h)
        out = {}
        for mode, ep, counters in (("defer", 2, False), ("inlane", 0, False), ("exact", 2, True)):
            r.set_exact_pass(ep)
            hist = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda")
            cnt = torch.zeros(len(vrt.COUNTER_NAMES), dtype=torch.int64, device="cuda")
            seq = []
            for t in range(3):
                p = vrt.textured_params(vrt.default_params(R, T, time=float(t + 1)), atlas)
                r.render_temporal_rows_async(cam, p, 0.5, 0, h, 1, hist.data_ptr(), hist.data_ptr(),
                                             d_counters=cnt.data_ptr() if counters else 0,
                                             stream=torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                seq.append(hist.cpu().numpy().copy())
            out[mode] = seq
    for t in range(3):
        assert np.array_equal(out["defer"][t], out["exact"][t]), f"deferred, frame {t}"
        assert np.array_equal(out["inlane"][t], out["exact"][t]), f"in-lane, frame {t}"


LONE = [("glass_cube", 128, 1920, 1080, 1, 2), ("terrain", 128, 3840, 2160, 4, 2)]


@pytest.mark.parametrize("case", LONE, ids=[f"{c[0]}_{c[2]}x{c[3]}" for c in LONE])
def test_synchronous_frames_deferred(built, case):
    """vrt_render_frame renders a glass-heavy volume's frame, or a frame of >= 8 rounds of
    resident waves, as one deferred launch (certified pass + the exact pass's short-band
    instance); the frames must equal the in-lane path's (exact pass off) and the counted exact
    instance's, frame after frame through the history (u_Alpha 0.5 and 1)."""
    scene, n, w, h, R, T = case
    vox = vrt.build_scene(scene, n)
    cam = vrt.make_camera(w, h)
    got = {}
    for mode in (1, 0):
        with vrt.Renderer(0) as r:
            r.upload_volume(vox, n)
            r.set_exact_pass(mode)
            got[mode] = [r.render_frame(cam, vrt.default_params(R, T, time=float(t + 1)), a)[0]
                         for t, a in enumerate((1.0, 0.5, 1.0))]
    with vrt.Renderer(0) as r:
        r.upload_volume(vox, n)
        ref = [r.render_frame(cam, vrt.default_params(R, T, time=float(t + 1)), a, counters=True)[0]
               for t, a in enumerate((1.0, 0.5, 1.0))]
    for k in range(3):
        assert np.array_equal(got[1][k], ref[k]), f"deferred, frame {k}"
        assert np.array_equal(got[0][k], ref[k]), f"in-lane, frame {k}"
