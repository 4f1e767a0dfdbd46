"""GPU parity of the fused temporal filter + RGB8 framebuffer epilogue (SURVEY §8f row 1;
temporal.glsl:18, main.cpp:363-393,417-421, FrameBuffer.cpp:8) through the C-ABI.

Contract:
  - the blend is bit-exact: the device's filtered bytes equal oracle.temporal_from_raw() applied
    to the device's own quantised ray-trace bytes and the same history
  - the quantised ray-trace bytes equal the oracle's quantisation of the oracle's float colour,
    except where that colour lies within COLOR_TOL (the float-colour contract, 1e-4) of a
    rounding boundary of x*255; there a 1-LSB difference is allowed (and counted)
"""
import numpy as np
import pytest
import torch

import oracle
import voxelraytracer_amd as vrt

pytestmark = pytest.mark.gpu

COLOR_TOL = 1e-4


@pytest.fixture(scope="module")
def renderer(built):
    r = vrt.Renderer(0)
    yield r
    r.close()


def check_raw(raw_g, rgba_o):
    """Device RGB8 bytes vs the oracle's float colour quantised by the oracle."""
    raw_o, _ = oracle.temporal(rgba_o, np.zeros(rgba_o.shape, np.uint8), 1.0)
    diff = raw_g[..., :3].astype(np.int16) - raw_o[..., :3].astype(np.int16)
    bad = diff != 0
    assert np.abs(diff).max(initial=0) <= 1
    if bad.any():   # only where the oracle colour is within COLOR_TOL of a .5 boundary
        x = np.clip(rgba_o[..., :3][bad], 0, 1).astype(np.float64) * 255.0
        assert np.all(np.abs(x - np.floor(x) - 0.5) <= COLOR_TOL * 255.0)
    assert np.all(raw_g[..., 3] == 255)
    return int(bad.sum())


def scene(renderer, name, n, w, h, R, T, **kw):
    vox = vrt.build_scene(name, n)
    renderer.upload_volume(vox, n)
    cam = vrt.make_camera(w, h)
    return vox, cam, vrt.default_params(R, T, **kw)


@pytest.mark.parametrize("name,n,w,h,R,T,alpha,extra", [
    ("glass_cube", 32, 160, 120, 1, 2, 1.0, {}),
    ("terrain", 64, 192, 108, 4, 2, 0.3, dict(ray_noise=0.02, time=5.0)),
    ("refraction", 128, 320, 180, 4, 4, 0.75, {}),
    ("glass_cube", 16, 64, 48, 4, 4, 0.0, dict(reflection_noise=0.1, time=2.0)),
])
def test_temporal_band_parity(renderer, name, n, w, h, R, T, alpha, extra):
    vox, cam, p = scene(renderer, name, n, w, h, R, T, **extra)
    rng = np.random.default_rng(n + w)
    prev = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    d_prev = torch.from_numpy(prev).cuda()
    d_cur = torch.empty((h, w, 4), dtype=torch.uint8, device="cuda")
    d_raw = torch.empty((h, w, 4), dtype=torch.uint8, device="cuda")
    renderer.render_temporal_rows_async(cam, p, alpha, 0, h, 1, d_prev.data_ptr(),
                                        d_cur.data_ptr(), d_raw.data_ptr())
    torch.cuda.synchronize()
    raw_g, cur_g = d_raw.cpu().numpy(), d_cur.cpu().numpy()
    assert np.array_equal(cur_g, oracle.temporal_from_raw(raw_g, prev, alpha))
    rgba_o, _, _ = oracle.render(cam, vox, n, p, threads=16)
    check_raw(raw_g, rgba_o)
    # the float path's colour quantises to the same bytes (same kernel, same colour)
    rgba_g, _, _ = renderer.render(cam, p, want_hits=False)
    raw_f, _ = oracle.temporal(rgba_g, prev, 1.0)
    assert np.array_equal(raw_f, raw_g)


def test_temporal_in_place_and_cyclic_bands(renderer):
    """History aliased with the output (in-place update) and cyclic row bands (multi-GPU
    tiling) reproduce the full-frame result exactly."""
    vox, cam, p = scene(renderer, "terrain", 32, 96, 60, 4, 2)
    h, w, alpha = 60, 96, 0.4
    prev = np.random.default_rng(1).integers(0, 256, (h, w, 4), dtype=np.uint8)
    ref = torch.empty((h, w, 4), dtype=torch.uint8, device="cuda")
    renderer.render_temporal_rows_async(cam, p, alpha, 0, h, 1,
                                        torch.from_numpy(prev).cuda().data_ptr(), ref.data_ptr())
    k = 3
    bands = torch.from_numpy(np.ascontiguousarray(
        np.stack([prev[r::k] for r in range(k)]))).cuda()          # [k, h/k, w, 4]
    for r in range(k):
        renderer.render_temporal_rows_async(cam, p, alpha, r, h // k, k, bands[r].data_ptr(),
                                            bands[r].data_ptr())   # in place
    torch.cuda.synchronize()
    frame = bands.permute(1, 0, 2, 3).reshape(h, w, 4).cpu().numpy()
    assert np.array_equal(frame, ref.cpu().numpy())


def test_frame_loop_history_and_reset(renderer):
    """vrt_render_frame keeps main.cpp's two history FBOs: frame k blends against frame k-1's
    output; the history starts black; vrt_history_reset makes the last ray-traced frame the
    history (key F)."""
    vox, cam, p = scene(renderer, "refraction", 32, 128, 72, 4, 4)
    h, w = 72, 128
    d_raw = torch.empty((h, w, 4), dtype=torch.uint8, device="cuda")
    zeros = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda")
    renderer.render_temporal_rows_async(cam, p, 1.0, 0, h, 1, zeros.data_ptr(), d_raw.data_ptr())
    torch.cuda.synchronize()
    raw = d_raw.cpu().numpy()             # the frame's quantised colour (deterministic)
    f1, st = renderer.render_frame(cam, p, 0.5, counters=True)
    assert np.array_equal(f1, oracle.temporal_from_raw(raw, np.zeros_like(raw), 0.5))
    f2, _ = renderer.render_frame(cam, p, 0.5)
    assert np.array_equal(f2, oracle.temporal_from_raw(raw, f1, 0.5))
    renderer.history_reset()
    f3, _ = renderer.render_frame(cam, p, 0.0)   # alpha 0: output = history = last raw frame
    assert np.array_equal(f3, raw)
    rgba_o, _, cnt_o = oracle.render(cam, vox, 32, p, threads=16)
    check_raw(raw, rgba_o)
    for k in oracle.COUNTER_NAMES:
        assert st[k] == cnt_o[k], k
    # a new image size restarts from a black history
    cam2 = vrt.make_camera(64, 36)
    g, _ = renderer.render_frame(cam2, p, 0.5)
    d2 = torch.empty((36, 64, 4), dtype=torch.uint8, device="cuda")
    z2 = torch.zeros_like(d2)
    renderer.render_temporal_rows_async(cam2, p, 1.0, 0, 36, 1, z2.data_ptr(), d2.data_ptr())
    torch.cuda.synchronize()
    r2 = d2.cpu().numpy()
    assert np.array_equal(g, oracle.temporal_from_raw(r2, np.zeros_like(r2), 0.5))


def test_temporal_errors(renderer):
    vox, cam, p = scene(renderer, "glass_cube", 16, 8, 8, 1, 2)
    d = torch.zeros((8, 8, 4), dtype=torch.uint8, device="cuda")
    with pytest.raises(vrt.VrtError):
        renderer.render_temporal_rows_async(cam, p, 1.0, 0, 8, 1, 0, d.data_ptr())
    with pytest.raises(vrt.VrtError):
        renderer.render_temporal_rows_async(cam, p, 1.0, 4, 8, 1, d.data_ptr(), d.data_ptr())


@pytest.mark.parametrize("k", [2, 3])
def test_pitched_bands_write_the_frame_in_place(renderer, k):
    """ABI v4 pitched forms: band r (rows r, r+k, ...) written through pitch = k*W straight into
    a full frame, filtered in place against the same rows, equals the whole-frame render; the
    float form likewise; a pitch below the width is rejected."""
    w, h = 96, 72
    _, cam, p = scene(renderer, "refraction", 32, w, h, 4, 4, ray_noise=0.02, time=3.0)
    rng = np.random.default_rng(k)
    prev = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    ref = torch.from_numpy(prev).cuda()
    renderer.render_temporal_rows_async(cam, p, 0.6, 0, h, 1, ref.data_ptr(), ref.data_ptr())
    frame = torch.from_numpy(prev).cuda()
    raw = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda")
    for r in range(k):
        renderer.render_temporal_rows_async(cam, p, 0.6, r, h // k, k, frame[r].data_ptr(),
                                            frame[r].data_ptr(), raw[r].data_ptr(), pitch=k * w)
    fref = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
    renderer.render_rows_async(cam, p, 0, h, 1, fref.data_ptr())
    fpart = torch.full((h, w, 4), -1.0, dtype=torch.float32, device="cuda")
    for r in range(k):
        renderer.render_rows_async(cam, p, r, h // k, k, fpart[r].data_ptr(), pitch=k * w)
    torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy(), ref.cpu().numpy())
    assert np.all(raw.cpu().numpy()[..., 3] == 255)   # every raw row was written too
    assert np.array_equal(fpart.cpu().numpy(), fref.cpu().numpy())
    with pytest.raises(vrt.VrtError):
        renderer.render_temporal_rows_async(cam, p, 1.0, 0, h, 1, frame.data_ptr(),
                                            frame.data_ptr(), pitch=w - 1)
