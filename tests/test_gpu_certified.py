"""GPU: the stats-free colour-only kernel instance (certified walks, exact fallback) renders the
same image, bit for bit, as the stats instance (exact walks, itself checked against the oracle in
test_gpu_parity.py).

The certified walk (DESIGN.md §6 "Certified walks") returns a primary walk's outcome (miss, or the
first event's byte and face axis) and a shadow walk's blocked bit without replaying the exact
walk's float state, and falls back to the exact walk whenever a rounding of the exact walk could
change the outcome. These cases aim at exactly those roundings: cameras on lattice points and
half-integers, rays along lattice diagonals (ties), faces hit at their edges, rays grazing the
volume's faces and the GL_REPEAT plane N, and random sparse scenes with every byte value.
"""
import numpy as np
import pytest
import torch

import voxelraytracer_amd as vrt

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["trees", "no_trees"])
def renderer(built, request):
    r = vrt.Renderer(0)
    r.set_certified(1)   # every case below exercises the certified walks, whatever the scene
    # ... with certified bounce trees forced on (every glass pixel tries one) and off
    r.tree_mode = 2 if request.param == "trees" else 0
    r.set_cert_trees(r.tree_mode)
    yield r
    r.close()


def stats_free(renderer, cam, p, h, w):
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    renderer.render_rows_async(cam, p, 0, h, 1, out.data_ptr(), 0, 0)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def check_same(renderer, vox, n, w, h, R, T, **kw):
    renderer.upload_volume(vox, n)
    cam = vrt.make_camera(w, h, **{k: kw.pop(k) for k in ("pos", "rot") if k in kw})
    p = vrt.default_params(R, T, **kw)
    exact, _, _ = renderer.render(cam, p)
    fast = stats_free(renderer, cam, p, h, w)
    bad = np.argwhere(np.any(exact.view(np.uint32) != fast.view(np.uint32), axis=-1))
    assert bad.size == 0, f"{len(bad)} pixels differ, first {bad[:5].tolist()}"


@pytest.mark.parametrize("scene,n,w,h,R,T", [
    ("glass_cube", 128, 1920, 1080, 1, 2), ("terrain", 128, 1920, 1080, 4, 2),
    ("refraction", 128, 1920, 1080, 4, 4), ("terrain", 512, 3840, 2160, 4, 2),
    ("terrain", 64, 320, 180, 4, 4), ("glass_cube", 16, 400, 400, 1, 2)])
def test_certified_baseline_frames(renderer, scene, n, w, h, R, T):
    check_same(renderer, vrt.build_scene(scene, n), n, w, h, R, T)


LATTICE = [
    # camera positions relative to the volume centre (world = pos + N/2) and rotations (deg)
    ((0.0, 0.0, 0.0), (0.0, 0.0, 0.0)),
    ((0.0, 0.0, 0.0), (-35.26439, 45.0, 0.0)),      # the central ray along (1,1,1)/sqrt 3
    ((0.5, 0.5, 0.5), (-35.26439, 45.0, 0.0)),
    ((0.0, 0.0, 0.0), (0.0, 45.0, 0.0)),            # x = z diagonal: edge ties
    ((1.0, -2.0, 3.0), (-45.0, 0.0, 0.0)),
    ((0.0, 0.0, 0.0), (-90.0, 0.0, 0.0)),           # straight down: tiny components
    ((0.25, 0.75, -0.5), (-30.0, 135.0, 0.0)),
    ((0.0, 0.0, 0.0), (0.0, 180.0, 0.0)),
]


@pytest.mark.parametrize("scene,n", [("terrain", 32), ("refraction", 32), ("glass_cube", 16),
                                     ("terrain", 128)])
@pytest.mark.parametrize("li", range(len(LATTICE)))
def test_certified_lattice_cameras(renderer, scene, n, li):
    pos, rot = LATTICE[li]
    check_same(renderer, vrt.build_scene(scene, n), n, 97, 65, 4, 4, pos=pos, rot=rot)


def random_scene(n, density, seed):
    rng = np.random.default_rng(seed)
    vox = np.zeros((n, n, n), np.uint8)
    m = rng.random((n, n, n)) < density
    vox[m] = rng.choice(np.array([1, 2, 3, 7, 200, 255], np.uint8), size=int(m.sum()))
    # solid slabs and single-voxel pillars: faces, edges and corners at lattice positions
    vox[:, : n // 8, :] = 1
    vox[n // 2, :, n // 2] = 3
    vox[: n // 4, n // 2, : n // 4] = 255
    return vox.reshape(-1)


@pytest.mark.parametrize("seed", range(6))
def test_certified_random_scenes(renderer, seed):
    rng = np.random.default_rng(100 + seed)
    n = [16, 32, 64, 32, 128, 16][seed]
    vox = random_scene(n, [0.002, 0.01, 0.03, 0.0, 0.001, 0.05][seed], seed)
    for _ in range(3):
        pos = tuple(float(x) for x in np.round(rng.uniform(-n / 3, n / 3, 3) * 2) / 2)
        rot = (float(rng.choice([-90, -45, -35.26439, -20, 0, 10])),
               float(rng.choice([0, 45, 90, 135, 180, 225, 270, 315, 33.3])), 0.0)
        check_same(renderer, vox, n, 80, 60, 2, 2, pos=pos, rot=rot)


def test_certified_camera_outside_and_noise(renderer):
    """Cameras outside the volume (exact path) and ray noise > 0 (direction hashing)."""
    n = 32
    vox = vrt.build_scene("terrain", n)
    check_same(renderer, vox, n, 96, 64, 4, 2, pos=(0.0, 40.0, 0.0), rot=(-60.0, 30.0, 0.0))
    check_same(renderer, vox, n, 96, 64, 4, 2, ray_noise=0.05, time=3.0)
    check_same(renderer, vox, n, 96, 64, 4, 2, max_ray_length=20.0)
    g = vrt.build_scene("glass_cube", n)
    check_same(renderer, g, n, 96, 64, 4, 4, reflection_noise=0.05, time=2.0)
    check_same(renderer, g, n, 96, 64, 4, 4, refraction_noise=0.01, time=2.0)
    check_same(renderer, g, n, 96, 64, 1, 8, max_ray_length=40.0)


@pytest.mark.parametrize("seed", range(4))
def test_certified_glass_scenes(renderer, seed):
    """Glass everywhere: bounce stacks, in-volume refraction, total internal reflection."""
    rng = np.random.default_rng(200 + seed)
    n = [16, 32, 64, 32][seed]
    vox = np.zeros((n, n, n), np.uint8)
    m = rng.random((n, n, n)) < [0.05, 0.02, 0.01, 0.1][seed]
    vox[m] = rng.choice(np.array([2, 2, 2, 1, 3], np.uint8), size=int(m.sum()))
    vox[n // 4: n // 2, n // 4: n // 2, n // 4: n // 2] = 2   # a solid glass block
    vox[:, :2, :] = 1
    vox = vox.reshape(-1)
    for _ in range(3):
        pos = tuple(float(x) for x in np.round(rng.uniform(-n / 3, n / 3, 3) * 2) / 2)
        rot = (float(rng.choice([-60, -45, -35.26439, -20, 0])),
               float(rng.choice([0, 45, 90, 135, 200, 33.3])), 0.0)
        check_same(renderer, vox, n, 72, 54, 4, 4, pos=pos, rot=rot)


def test_certified_modes(renderer):
    """Automatic mode: on unless glass is > 1/8 of the non-empty voxels (the glass cube), and with
    certified bounce trees (ABI v15: automatic, i.e. for exactly those volumes, or always) on for
    every volume. Every mode, with and without trees, renders the same image."""
    try:
        for scene, n, auto in (("glass_cube", 64, False), ("refraction", 64, True), ("terrain", 128, True)):
            vox = vrt.build_scene(scene, n)
            renderer.upload_volume(vox, n)
            renderer.set_certified(0)
            for trees in (1, 2):
                renderer.set_cert_trees(trees)
                assert renderer.certified()
            renderer.set_cert_trees(0)
            assert renderer.certified() == auto, scene
            renderer.set_certified(-1)
            assert not renderer.certified()
            cam = vrt.make_camera(96, 64)
            p = vrt.default_params(4, 4)
            imgs = []
            for trees in (0, 1, 2):
                renderer.set_cert_trees(trees)
                for mode in (-1, 0, 1):
                    renderer.set_certified(mode)
                    imgs.append(stats_free(renderer, cam, p, 64, 96))
            for im in imgs[1:]:
                assert np.array_equal(imgs[0].view(np.uint32), im.view(np.uint32))
        with pytest.raises(vrt.VrtError):
            renderer.set_certified(2)
        with pytest.raises(vrt.VrtError):
            renderer.set_cert_trees(3)
    finally:
        renderer.set_certified(1)
        renderer.set_cert_trees(renderer.tree_mode)


@pytest.mark.parametrize("seed", range(4))
def test_certified_glass_slabs_continuations(renderer, seed):
    """Bounce stacks through glass slabs and rods: refraction rays cross the glass and leave it by
    in-volume refraction (the certified march continuation, with the refracted axis' plane offset),
    at lattice-aligned cameras and views along lattice diagonals; thick slabs give total internal
    reflection."""
    n = [32, 64, 32, 64][seed]
    vox = np.zeros((n, n, n), np.uint8)
    vox[:, : n // 8, :] = 1                                      # floor
    t = [1, 2, 3, 5][seed]
    vox[n // 3: n // 3 + t, n // 8: n // 2, n // 4: 3 * n // 4] = 2   # upright slab, thickness t
    vox[n // 4: 3 * n // 4, n // 2: n // 2 + t, n // 2] = 2            # a rod along x
    vox[2 * n // 3, n // 8: n // 3, n // 5: n // 5 + t] = 3            # an opaque post
    if seed % 2:
        vox[n // 2: n // 2 + 4, n // 3: n // 3 + 4, n // 2: n // 2 + 4] = 2   # a glass block
    vox = vox.reshape(-1)
    for pos, rot in LATTICE[:6]:
        check_same(renderer, vox, n, 64, 48, 4, 4, pos=pos, rot=rot)
    check_same(renderer, vox, n, 64, 48, 4, 4, pos=(0.5, 2.0, -6.0), rot=(-15.0, 20.0, 0.0),
               refraction_noise=0.02, time=1.5)


@pytest.mark.parametrize("scene,n,R,T", [("refraction", 128, 4, 4), ("terrain", 128, 4, 2),
                                         ("glass_cube", 64, 1, 2)])
def test_certified_random_poses(renderer, scene, n, R, T):
    """128 random camera poses inside and around each BASELINE scene (positions within ±N/2 of the
    centre, any yaw, pitch in ±80 degrees, random sun time): every certified frame equals the
    exact instance's, pixel for pixel."""
    rng = np.random.default_rng(sum(map(ord, scene)) + n)
    vox = vrt.build_scene(scene, n)
    renderer.upload_volume(vox, n)
    w, h = 256, 144
    for k in range(128):
        pos = tuple(float(x) for x in rng.uniform(-0.5 * n, 0.5 * n, 3))
        rot = (float(rng.uniform(-80, 80)), float(rng.uniform(-180, 180)), 0.0)
        cam = vrt.make_camera(w, h, pos=pos, rot=rot)
        p = vrt.default_params(R, T, time=float(k + 1),
                               sun_dir=vrt.sun_dir(float(rng.uniform(0.0, 50.0))))
        exact, _, _ = renderer.render(cam, p)
        fast = stats_free(renderer, cam, p, h, w)
        bad = np.argwhere(np.any(exact.view(np.uint32) != fast.view(np.uint32), axis=-1))
        assert bad.size == 0, f"pose {k} {pos} {rot}: {len(bad)} pixels differ, first {bad[:5].tolist()}"
