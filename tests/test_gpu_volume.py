"""The kernel's device volume format (GPU): per direction octant a padded (N+1)^3 u16 = voxel |
G << 8, with plane N a copy of plane 0 (GL_REPEAT) and G the forward skip distance of the octant
(G(v) = F(v - s) - 1, F = edge of the largest empty in-volume cube anchored at a voxel and
extending along the octant's step s) — checked against a brute-force NumPy transform; for
N = 1024 one volume with the centred Chebyshev distance (tested at small N through the same
reference). G drives the empty-space step skipping, so an over-estimate would skip geometry
(DESIGN.md §6)."""
import numpy as np
import pytest

import voxelraytracer_amd as vrt

pytestmark = pytest.mark.gpu
CAP = 64  # kDistCap (VRT_DIST_CAP) of csrc/vrt_render.hip
FWD_CAP = 128  # kFwdCap (VRT_FWD_CAP)


def forward_reference(vox, n, octant):
    """G of `octant` ([z][y][x] n^3) by brute force: in coordinates flipped so that the octant's
    step is +1 on every axis, F(v) = the largest E with v + E <= n and the box [v, v+E-1]^3
    empty (prefix-sum box counts), G(v) = F(v - 1) - 1 clamped at 0 (0 on the low faces)."""
    sl = tuple(slice(None, None, -1) if octant >> a & 1 else slice(None) for a in (2, 1, 0))
    occ = (vox.reshape(n, n, n) != 0)[sl].astype(np.int64)
    c = np.zeros((n + 1,) * 3, np.int64)
    c[1:, 1:, 1:] = occ.cumsum(0).cumsum(1).cumsum(2)
    f = np.zeros((n, n, n), np.int64)
    for e in range(1, min(FWD_CAP, n) + 1):
        m = n - e + 1   # anchors with v + e <= n on every axis
        i0 = np.arange(m)
        z0, y0, x0 = i0[:, None, None], i0[None, :, None], i0[None, None, :]
        z1, y1, x1 = z0 + e, y0 + e, x0 + e
        cnt = (c[z1, y1, x1] - c[z0, y1, x1] - c[z1, y0, x1] - c[z1, y1, x0] + c[z0, y0, x1]
               + c[z0, y1, x0] + c[z1, y0, x0] - c[z0, y0, x0])
        sub = f[:m, :m, :m]
        f[:m, :m, :m] = np.where(cnt == 0, e, sub)
    g = np.zeros((n, n, n), np.int64)
    g[1:, 1:, 1:] = np.maximum(f[:-1, :-1, :-1] - 1, 0)
    return g[sl]


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
        vols = r.debug_packed_volume()   # [octant][z][y][x], 8 x (n+1)^3
    assert vols.shape[0] == 8
    v = vox.reshape(n, n, n)
    for o, packed in enumerate(vols):
        assert np.array_equal(packed[:n, :n, :n] & 0xFF, v)
        assert np.array_equal(packed[n, :n, :n] & 0xFF, v[0])        # plane z = N repeats z = 0
        assert np.array_equal(packed[:n, n, :n] & 0xFF, v[:, 0])
        assert np.array_equal(packed[:n, :n, n] & 0xFF, v[:, :, 0])
        assert np.all(packed[n] >> 8 == 0) and np.all(packed[:, n] >> 8 == 0)
        assert np.all(packed[:, :, n] >> 8 == 0)
        assert np.array_equal(packed[:n, :n, :n] >> 8, forward_reference(vox, n, o)), o
        # the guarantee the skip walk relies on, stated directly: the box from one voxel behind
        # to G - 1 voxels ahead (along the octant's step) holds no non-empty voxel
        g = packed[:n, :n, :n] >> 8
        s = [(-1 if o >> a & 1 else 1) for a in range(3)]   # x, y, z steps
        zz, yy, xx = np.nonzero(g >= 1)
        for q in range(0, len(zz), max(1, len(zz) // 300)):
            k, j, i, e = zz[q], yy[q], xx[q], int(g[zz[q], yy[q], xx[q]])
            lo = [min(c - sc, c + (e - 1) * sc) for c, sc in zip((i, j, k), s)]
            hi = [max(c - sc, c + (e - 1) * sc) for c, sc in zip((i, j, k), s)]
            assert min(lo) >= 0 and max(hi) < n
            assert not v[lo[2]:hi[2] + 1, lo[1]:hi[1] + 1, lo[0]:hi[0] + 1].any()


@pytest.mark.parametrize("scene,n", [("terrain", 16), ("refraction", 32)])
def test_single_layout_centred_distance(built, scene, n):
    """The N = 1024 layout (one volume, centred Chebyshev D), forced at small N."""
    vox = vrt.build_scene(scene, n)
    with vrt.Renderer(0) as r:
        r.set_skip_layout(1)
        r.upload_volume(vox, n)
        vols = r.debug_packed_volume()
    assert vols.shape[0] == 1
    packed = vols[0]
    assert np.array_equal(packed[:n, :n, :n] & 0xFF, vox.reshape(n, n, n))
    assert np.all(packed[n] >> 8 == 0) and np.all(packed[:, n] >> 8 == 0)
    assert np.array_equal(packed[:n, :n, :n] >> 8, chebyshev_reference(vox, n))


@pytest.mark.parametrize("scene,n,w,h,rt", [("terrain", 64, 160, 90, (4, 2)),
                                            ("refraction", 64, 160, 90, (4, 4)),
                                            ("glass_cube", 32, 128, 96, (1, 2))])
def test_layouts_render_identically(built, scene, n, w, h, rt):
    """Octant and single (centred) layouts skip different steps but replay the same walk: images,
    hit records and every counter are identical."""
    vox = vrt.build_scene(scene, n)
    cam = vrt.make_camera(w, h)
    p = vrt.default_params(*rt)
    res = []
    for layout in (8, 1):
        with vrt.Renderer(0) as r:
            r.set_skip_layout(layout)
            r.upload_volume(vox, n)
            res.append(r.render(cam, p))
    (ra, ha, sa), (rb, hb, sb) = res
    assert np.array_equal(ra.view(np.uint32), rb.view(np.uint32))
    assert np.array_equal(ha, hb)
    assert {k: v for k, v in sa.items() if k != "kernel_ms"} == \
        {k: v for k, v in sb.items() if k != "kernel_ms"}


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
