"""GPU: the heavy-first tile order (vrt_set_tile_order, DESIGN.md §6 "Tile order") changes only
which workgroup renders which tile and when: every tile is rendered exactly once, so frames are
bit-identical with and without it — over consecutive frames (the order of frame k comes from frame
k - 1), for interleaved bands on two streams, for geometry changes, and for the in-place temporal
filter with alpha < 1 (a tile rendered twice would blend twice)."""
import numpy as np
import pytest
import torch

import voxelraytracer_amd as vrt

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def renderer(built):
    r = vrt.Renderer(0)
    yield r
    r.set_tile_order(1)
    r.close()


def frames(renderer, cam, p, h, w, n_frames, bands=((0, 1),), streams=None):
    """n_frames stats-free float frames, each rendered as the given (row0, row_step) bands (one
    stream per band); returns the list of frames."""
    out = []
    devs = streams or [torch.cuda.current_stream()] * len(bands)
    for _ in range(n_frames):
        img = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
        for st in devs:
            st.wait_stream(torch.cuda.current_stream())
        for (row0, step), st in zip(bands, devs):
            rows = (h - row0 + step - 1) // step
            with torch.cuda.stream(st):
                renderer.render_rows_async(cam, p, row0, rows, step, img[row0:].data_ptr(), 0, 0,
                                           st.cuda_stream, pitch=w * step)
        torch.cuda.synchronize()
        out.append(img.cpu().numpy())
    return out


def same(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("scene,n,w,h,R,T", [("refraction", 128, 480, 270, 4, 4),
                                             ("glass_cube", 64, 320, 200, 1, 2),
                                             ("terrain", 64, 256, 144, 4, 2)])
def test_tile_order_frames_identical(renderer, scene, n, w, h, R, T):
    renderer.upload_volume(vrt.build_scene(scene, n), n)
    cam = vrt.make_camera(w, h)
    p = vrt.default_params(R, T)
    exact, _, _ = renderer.render(cam, p)   # stats instance: exact walks, dispatch order
    renderer.set_tile_order(2)
    for k, img in enumerate(frames(renderer, cam, p, h, w, 5)):
        assert same(img, exact), f"frame {k}"
    renderer.set_tile_order(False)
    assert same(frames(renderer, cam, p, h, w, 1)[0], exact)
    renderer.set_tile_order(2)


def test_tile_order_bands_streams_and_geometry(renderer):
    n = 128
    renderer.upload_volume(vrt.build_scene("refraction", n), n)
    p = vrt.default_params(4, 4)
    renderer.set_tile_order(2)
    s2 = [torch.cuda.Stream(), torch.cuda.Stream()]
    for w, h in ((400, 240), (416, 240), (400, 240), (200, 120)):
        cam = vrt.make_camera(w, h)
        exact, _, _ = renderer.render(cam, p)
        for k, img in enumerate(frames(renderer, cam, p, h, w, 4, bands=((0, 2), (1, 2)), streams=s2)):
            assert same(img, exact), f"{w}x{h} frame {k}"
        # a moving camera: the order recorded for one view is only a hint for the next
        cam2 = vrt.make_camera(w, h, pos=(3.0, 1.0, -2.0), rot=(-20.0, 30.0, 0.0))
        exact2, _, _ = renderer.render(cam2, p)
        assert same(frames(renderer, cam2, p, h, w, 1, bands=((0, 2), (1, 2)), streams=s2)[0], exact2)


def test_tile_order_temporal_in_place(renderer):
    """alpha 0.5 in place (prev aliases cur): each frame's result depends on every tile being
    filtered exactly once."""
    n, w, h = 128, 320, 180
    renderer.upload_volume(vrt.build_scene("refraction", n), n)
    cam = vrt.make_camera(w, h)
    p = vrt.default_params(4, 4)
    runs = []
    for on in (0, 2):
        renderer.set_tile_order(on)
        hist = torch.zeros((h, w), dtype=torch.int32, device="cuda")
        seq = []
        for _ in range(5):
            renderer.render_temporal_rows_async(cam, p, 0.5, 0, h, 1, hist.data_ptr(), hist.data_ptr(),
                                                0, 0, 0, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            seq.append(hist.cpu().numpy().copy())
        runs.append(seq)
    for k, (a, b) in enumerate(zip(*runs)):
        assert np.array_equal(a, b), f"frame {k}"
    assert not np.array_equal(runs[1][0], runs[1][-1])   # the blend did accumulate


def test_tile_order_switch(renderer):
    assert renderer._lib.vrt_set_tile_order(renderer._h, 3) == vrt.abi.VRT_ERR_INVALID
    assert renderer._lib.vrt_set_tile_order(renderer._h, -1) == vrt.abi.VRT_ERR_INVALID
    renderer.set_tile_order(2)


def test_tile_order_slot_recycling(renderer):
    """More (band geometry, stream) pairs than the pool's 8 slots, on three streams in turn: slots
    are recycled across streams (the new stream waits for the old one on the device) and every
    frame still equals the exact instance's."""
    n, w, h = 128, 256, 160
    renderer.upload_volume(vrt.build_scene("refraction", n), n)
    p = vrt.default_params(4, 4)
    renderer.set_tile_order(2)
    cam = vrt.make_camera(w, h)
    exact, _, _ = renderer.render(cam, p)
    streams = [torch.cuda.Stream() for _ in range(3)]
    for rnd in range(3):
        for k in range(1, 5):   # k interleaved bands: 1 + 2 + 3 + 4 = 10 geometries per round
            bands = tuple((r, k) for r in range(k))
            sts = [streams[(rnd + i) % 3] for i in range(k)]
            img = frames(renderer, cam, p, h, w, 1, bands=bands, streams=sts)[0]
            assert same(img, exact), f"round {rnd}, {k} bands"


def test_tile_order_graph_capture(renderer):
    """A launch captured into a HIP graph uses dispatch order (a replayed node cannot rotate the
    order state); replays equal the exact instance."""
    n, w, h = 128, 240, 136
    renderer.upload_volume(vrt.build_scene("refraction", n), n)
    p = vrt.default_params(4, 4)
    renderer.set_tile_order(2)
    cam = vrt.make_camera(w, h)
    exact, _, _ = renderer.render(cam, p)
    img = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # warm the stream outside the capture (the order slot exists)
        renderer.render_rows_async(cam, p, 0, h, 1, img.data_ptr(), 0, 0, s.cuda_stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        renderer.render_rows_async(cam, p, 0, h, 1, img.data_ptr(), 0, 0,
                                   torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        img.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert same(img.cpu().numpy(), exact)


def test_tile_order_band_beyond_the_pool(renderer):
    """A band of more tiles than a pool slot holds (131 072: here 7680 x 4320 = 259 200 tiles in
    one launch) renders in dispatch order; the frame equals the exact instance's."""
    n, w, h = 128, 7680, 4320
    renderer.upload_volume(vrt.build_scene("refraction", n), n)
    p = vrt.default_params(4, 4)
    renderer.set_tile_order(2)
    cam = vrt.make_camera(w, h)
    exact, _, _ = renderer.render(cam, p, want_hits=False)
    img = frames(renderer, cam, p, h, w, 2)
    for k, f in enumerate(img):
        assert same(f, exact), f"frame {k}"
