"""GPU: frame batches (vrt_render_temporal_batch_async, ABI v14). One launch renders the same band
of up to 8 frames, each with its own camera and u_Time, into its own RGBA8 buffer; the bytes must
equal the frames rendered one launch each, bit for bit — with the exact path in lane (tile order
forced on and off) and deferred to the exact pass, for whole frames and block-cyclic bands. Also
FrameTiler's batched lanes (bench.py's split frames) against single-frame rendering, and the
argument checks."""
import numpy as np
import pytest
import torch

import voxelraytracer_amd as vrt
from voxelraytracer_amd.tiles import FrameTiler, block_band_spec, row_pitch

pytestmark = pytest.mark.gpu


def cameras(w, h, nf):
    """nf different views (positions and angles) of the same image size."""
    return [vrt.make_camera(w, h, pos=(0.5 * f, 0.25 * f, -0.5 * f), rot=(-3.0 * f, 5.0 * f, 0.0))
            for f in range(nf)]


def params_for(R, T, nf):
    return [vrt.default_params(R, T, time=float(3 * f + 1), ray_noise=0.02) for f in range(nf)]


def singles(r, cams, ps, row0, rows, step, block):
    out = []
    for cam, p in zip(cams, ps):
        buf = torch.zeros((rows, cam.width), dtype=torch.int32, device="cuda")
        r.render_temporal_rows_async(cam, p, 1.0, row0, rows, step, buf.data_ptr(), buf.data_ptr(),
                                     stream=torch.cuda.current_stream().cuda_stream, row_block=block)
        out.append(buf)
    torch.cuda.synchronize()
    return [b.cpu().numpy() for b in out]


def batched(r, cams, ps, row0, rows, step, block):
    bufs = [torch.full((rows, cams[0].width), 7, dtype=torch.int32, device="cuda") for _ in cams]
    r.render_temporal_batch_async(cams, ps, row0, rows, step, [b.data_ptr() for b in bufs],
                                  stream=torch.cuda.current_stream().cuda_stream, row_block=block)
    torch.cuda.synchronize()
    return [b.cpu().numpy() for b in bufs]


@pytest.mark.parametrize("scene,n,w,h,R,T,nf,ranks,rank", [
    ("refraction", 128, 480, 270, 4, 4, 3, 1, 0),      # whole frames
    ("refraction", 128, 640, 360, 4, 4, 8, 8, 5),      # an 8-way block-cyclic band, 8 frames
    ("glass_cube", 64, 320, 200, 1, 2, 2, 2, 1),
    ("terrain", 64, 384, 216, 4, 2, 4, 4, 2),
    ("terrain", 64, 3840, 2160, 4, 2, 3, 1, 0),        # 3 x 64 800 tiles: two launches (2 + 1)
    ("refraction", 128, 3840, 2160, 4, 4, 7, 7, 0),    # 7 frames of a 7-way 4K band: one launch
])
def test_batch_equals_single_frames(built, scene, n, w, h, R, T, nf, ranks, rank):
    block = 16 if ranks > 1 else 1
    row0, rows, step = block_band_spec(rank, ranks, h, block) if ranks > 1 else (0, h, 1)
    cams, ps = cameras(w, h, nf), params_for(R, T, nf)
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene(scene, n), n)
        for mode, order in ((1, 1), (0, 2), (0, 0), (2, 1)):   # exact pass auto / in lane / forced
            r.set_exact_pass(mode)
            r.set_tile_order(order)
            ref = singles(r, cams, ps, row0, rows, step, block)
            for rep in range(3):   # repeated: the tile order and the exact-pass grid use history
                got = batched(r, cams, ps, row0, rows, step, block)
                for f in range(nf):
                    assert np.array_equal(got[f], ref[f]), f"mode {mode} order {order} rep {rep} frame {f}"
        assert not all(np.array_equal(ref[0], x) for x in ref[1:])   # the frames do differ


@pytest.mark.parametrize("ranks,rank", [(1, 0), (8, 2)])
def test_textured_batch_equals_single_frames(built, ranks, rank):
    """Textured frames (the reference's default build) in a batch: the textured frame-batch
    instances, deferred exact pass and in lane."""
    w, h, n, R, T, nf = 480, 270, 128, 4, 4, 4
    block = 16 if ranks > 1 else 1
    row0, rows, step = block_band_spec(rank, ranks, h, block) if ranks > 1 else (0, h, 1)
    atlas = vrt.make_atlas()
    cams = cameras(w, h, nf)
    ps = [vrt.textured_params(p, atlas) for p in params_for(R, T, nf)]
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene("refraction", n), n)
        for mode in (1, 2, 0):
            r.set_exact_pass(mode)
            ref = singles(r, cams, ps, row0, rows, step, block)
            for rep in range(2):
                got = batched(r, cams, ps, row0, rows, step, block)
                for f in range(nf):
                    assert np.array_equal(got[f], ref[f]), f"mode {mode} rep {rep} frame {f}"


def test_batch_argument_checks(built):
    w, h = 64, 32
    cams, ps = cameras(w, h, 2), params_for(4, 4, 2)
    buf = [torch.zeros((h, w), dtype=torch.int32, device="cuda") for _ in range(9)]
    ptrs = [b.data_ptr() for b in buf]
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene("refraction", 32), 32)
        with pytest.raises(vrt.VrtError):   # 9 frames
            r.render_temporal_batch_async(cameras(w, h, 9), params_for(4, 4, 9), 0, h, 1, ptrs)
        with pytest.raises(ValueError):     # a params list shorter than the cameras
            r.render_temporal_batch_async(cams, ps[:1], 0, h, 1, ptrs[:2])
        with pytest.raises(ValueError):     # a raw-output list shorter than the cameras
            r.render_temporal_batch_async(cams, ps, 0, h, 1, ptrs[:2], d_raws=ptrs[:1])
        with pytest.raises(vrt.VrtError):   # different image sizes
            r.render_temporal_batch_async([cams[0], vrt.make_camera(w + 16, h)], ps, 0, h, 1, ptrs[:2])
        with pytest.raises(vrt.VrtError):   # a null output
            r.render_temporal_batch_async(cams, ps, 0, h, 1, [ptrs[0], 0])
        r.render_temporal_batch_async(cams, ps, 0, h, 1, ptrs[:2])   # and a valid one passes
        torch.cuda.synchronize()


def test_batch_with_per_frame_params(built):
    """ABI v15: frames whose params differ beyond u_Time (the day/night cycle's sun, main.cpp:346-
    348; here also the bounce limits and noise) share a batch call; the library splits them into
    launches of equal params, in order. Bytes equal one launch per frame."""
    w, h, nf = 320, 180, 6
    cams = cameras(w, h, nf)
    ps = params_for(4, 4, nf)
    for f in range(nf):   # the sun moves every frame; frames 3-4 also change the bounce limits
        ps[f].sun_dir = (vrt.abi.C.c_float * 3)(*vrt.sun_dir(45.0 + 0.5 * (f // 2)))
    ps[3].max_reflections = ps[4].max_reflections = 1
    ps[4].refraction_noise = 0.01
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene("refraction", 64), 64)
        for mode in (1, 2):
            r.set_exact_pass(mode)
            ref = singles(r, cams, ps, 0, h, 1, 1)
            got = batched(r, cams, ps, 0, h, 1, 1)
            for f in range(nf):
                assert np.array_equal(got[f], ref[f]), f"mode {mode} frame {f}"


@pytest.mark.parametrize("batch,lanes,frames", [(8, 4, 21), (4, 2, 9), (2, 3, 4)])
def test_frame_tiler_batches(built, batch, lanes, frames):
    """FrameTiler's batched lanes (bench.py's split frames): every frame returned equals the band
    rendered alone, including a partial last batch flushed by finish()."""
    n, w, h, ranks, rank, block = 128, 320, 180, 8, 3, 16
    cam = vrt.make_camera(w, h)
    p = vrt.default_params(4, 4)
    dev = torch.device("cuda", 0)
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene("refraction", n), n)

        def launch_batch(row0, rows, step, outs, pitch, sp, row_block=1):
            r.render_temporal_batch_async([cam] * len(outs), p, row0, rows, step, outs, None, sp,
                                          pitch=pitch, row_block=row_block)

        def render_band(*a, **k):
            raise AssertionError("a batched tiler launches batches only")

        tiler = FrameTiler(w, h, render_band, dev, dtype=torch.uint8, lanes=lanes, independent=True,
                           world=ranks, rank=rank, gather=False, row_block=block, batch=batch,
                           launch_batch=launch_batch)
        row0, rows, step = block_band_spec(rank, ranks, h, block)
        ref = torch.zeros((rows, w, 4), dtype=torch.uint8, device=dev)
        r.render_temporal_rows_async(cam, p, 1.0, row0, rows, step, ref.data_ptr(), ref.data_ptr(),
                                     stream=torch.cuda.current_stream().cuda_stream,
                                     pitch=row_pitch(ref), row_block=block)
        got = []
        for _ in range(frames):
            got.append(tiler.frame())
            if len(got) > lanes * batch:   # a returned band stays valid for lanes x batch frames
                got.pop(0)
        tiler.finish()
        torch.cuda.synchronize()
        assert tiler.k == frames and tiler.pending == 0
        for i, g in enumerate(got):
            assert torch.equal(g[:rows], ref), f"frame {i}"
