"""The kernel's device volume format (GPU): padded (N+1)^3 u16 = voxel | D << 8, with plane N a
copy of plane 0 (GL_REPEAT) and D the capped Chebyshev distance to the nearest non-empty voxel or
to the outside — checked against a brute-force NumPy transform. D drives the empty-space step
skipping, so an over-estimate would skip geometry."""
import numpy as np
import pytest

import voxelraytracer_amd as vrt

pytestmark = pytest.mark.gpu
CAP = 64  # kDistCap (VRT_DIST_CAP) of csrc/vrt_render.hip


def chebyshev_reference(vox, n):
    occ = np.zeros((n + 2,) * 3, bool)   # [z][y][x] with a non-empty border at -1 and n
    occ[0, :, :] = occ[-1, :, :] = occ[:, 0, :] = occ[:, -1, :] = occ[:, :, 0] = occ[:, :, -1] = True
    occ[1:-1, 1:-1, 1:-1] = vox.reshape(n, n, n) != 0
    d = np.full((n, n, n), CAP, np.int32)
    for r in range(CAP - 1, -1, -1):   # smallest r with a non-empty voxel in the (2r+1)^3 box
        k = 2 * r + 1
        # box-OR via cumulative sums
        c = np.pad(occ.astype(np.int32), ((1, 0), (1, 0), (1, 0))).cumsum(0).cumsum(1).cumsum(2)
        lo = 1 - r + 1   # index shift: occ index i+1 = voxel i, padded once more for cumsum
        hi = lo + k
        idx = np.arange(n)

        def box(a):
            z0, z1 = idx[:, None, None] + lo - 1, idx[:, None, None] + hi - 1
            y0, y1 = idx[None, :, None] + lo - 1, idx[None, :, None] + hi - 1
            x0, x1 = idx[None, None, :] + lo - 1, idx[None, None, :] + hi - 1
            z0, z1, y0, y1, x0, x1 = [np.clip(v, 0, n + 2) for v in (z0, z1, y0, y1, x0, x1)]
            return (a[z1, y1, x1] - a[z0, y1, x1] - a[z1, y0, x1] - a[z1, y1, x0] + a[z0, y0, x1]
                    + a[z0, y1, x0] + a[z1, y0, x0] - a[z0, y0, x0])

        d = np.where(box(c) > 0, r, d)
    return d


@pytest.mark.parametrize("scene,n", [("terrain", 16), ("glass_cube", 16), ("refraction", 32),
                                     ("terrain", 32)])
def test_packed_volume_layout_and_distance(built, scene, n):
    vox = vrt.build_scene(scene, n)
    with vrt.Renderer(0) as r:
        r.upload_volume(vox, n)
        packed = r.debug_packed_volume()   # [z][y][x], (n+1)^3
    v = vox.reshape(n, n, n)
    assert np.array_equal(packed[:n, :n, :n] & 0xFF, v)
    assert np.array_equal(packed[n, :n, :n] & 0xFF, v[0])        # plane z = N repeats z = 0
    assert np.array_equal(packed[:n, n, :n] & 0xFF, v[:, 0])
    assert np.array_equal(packed[:n, :n, n] & 0xFF, v[:, :, 0])
    assert np.all(packed[n] >> 8 == 0) and np.all(packed[:, n] >> 8 == 0)
    assert np.array_equal(packed[:n, :n, :n] >> 8, chebyshev_reference(vox, n))


@pytest.mark.parametrize("scene", ["terrain", "glass_cube", "refraction"])
@pytest.mark.parametrize("n", [16, 32, 64, 128])
def test_device_scene_builder_matches_host(built, scene, n):
    """vrt_build_scene_device (main.cpp:218-288 on the GPU) yields the same packed volume (voxel
    bytes + distance field) as uploading vrt_build_scene's host bytes, and the same frame."""
    with vrt.Renderer(0) as a, vrt.Renderer(0) as b:
        a.upload_volume(vrt.build_scene(scene, n), n)
        b.build_scene_device(scene, n)
        assert np.array_equal(a.debug_packed_volume(), b.debug_packed_volume())
        cam = vrt.make_camera(96, 54)
        p = vrt.default_params(4, 2)
        ra, _, _ = a.render(cam, p, want_hits=False)
        rb, _, _ = b.render(cam, p, want_hits=False)
        assert np.array_equal(ra.view(np.uint32), rb.view(np.uint32))


def test_device_scene_builder_512_terrain(built):
    with vrt.Renderer(0) as a, vrt.Renderer(0) as b:
        a.upload_volume(vrt.build_scene("terrain", 512), 512)
        b.build_scene_device("terrain", 512)
        assert np.array_equal(a.debug_packed_volume(), b.debug_packed_volume())
