"""GPU: block-cyclic bands (ABI v11, vrt_render_temporal_blocks_pitched_async /
vrt_render_blocks_pitched_async). Band row i is frame row row0 + (i // B) * row_step + i % B; every
rank's band of a k-way split must equal its rows of the whole frame bit for bit — certified pass
with the deferred exact pass, in-lane exact path (tile order), and the exact STATS instance —
including ragged splits (the last block short, bands of unequal height) and temporal frames that
read their band-local history."""
import numpy as np
import pytest
import torch

import voxelraytracer_amd as vrt
from voxelraytracer_amd.tiles import band_frame_rows, block_band_spec

pytestmark = pytest.mark.gpu


def band_frames(r, cam, R, T, alpha, row0, rows, step, block, exact_pass, n_frames=2, counters=False):
    r.set_exact_pass(exact_pass)
    w = cam.width
    hist = torch.zeros((rows, w, 4), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(len(vrt.COUNTER_NAMES), dtype=torch.int64, device="cuda")
    out = []
    for t in range(n_frames):
        p = vrt.default_params(R, T, time=float(t + 1))
        r.render_temporal_rows_async(cam, p, alpha, row0, rows, step, hist.data_ptr(), hist.data_ptr(),
                                     d_counters=cnt.data_ptr() if counters else 0,
                                     stream=torch.cuda.current_stream().cuda_stream, row_block=block)
        torch.cuda.synchronize()
        out.append(hist.cpu().numpy().copy())
    return out


CASES = [  # scene, n, w, h, R, T, world, block
    ("refraction", 128, 480, 270, 4, 4, 8, 8),
    ("terrain", 128, 384, 203, 4, 2, 3, 4),
    ("glass_cube", 64, 320, 180, 1, 2, 4, 8),
    ("refraction", 64, 256, 100, 4, 4, 16, 8),   # more ranks than blocks: empty bands
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}{c[1]}_{c[2]}x{c[3]}_k{c[6]}b{c[7]}" for c in CASES])
def test_block_bands_equal_the_whole_frame(built, case):
    scene, n, w, h, R, T, world, block = case
    vox = vrt.build_scene(scene, n)
    with vrt.Renderer(0) as r:
        r.upload_volume(vox, n)
        cam = vrt.make_camera(w, h)
        full = band_frames(r, cam, R, T, 0.5, 0, h, 1, 1, 1, counters=True)   # exact STATS instance
        for rank in range(world):
            row0, rows, step = block_band_spec(rank, world, h, block)
            if rows == 0:
                continue
            idx = band_frame_rows(row0, rows, step, block).numpy()
            for mode in (2, 0):   # deferred exact pass, in-lane exact path
                got = band_frames(r, cam, R, T, 0.5, row0, rows, step, block, mode)
                for k in range(2):
                    assert np.array_equal(got[k], full[k][idx]), (rank, mode, k)
            ref = band_frames(r, cam, R, T, 0.5, row0, rows, step, block, 1, counters=True)
            for k in range(2):
                assert np.array_equal(ref[k], full[k][idx]), (rank, "stats", k)


def test_block_band_float_output_and_arguments(built):
    """The float form, and the argument checks: row_block a power of two <= 64, blocks that do
    not overlap, the last row inside the image."""
    n, w, h = 64, 160, 90
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene("refraction", n), n)
        cam = vrt.make_camera(w, h)
        p = vrt.default_params(4, 4)
        st = torch.cuda.current_stream().cuda_stream
        full = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
        r.render_rows_async(cam, p, 0, h, 1, full.data_ptr(), stream=st)
        row0, rows, step = block_band_spec(1, 3, h, 8)
        band = torch.zeros((rows, w, 4), dtype=torch.float32, device="cuda")
        r.render_rows_async(cam, p, row0, rows, step, band.data_ptr(), stream=st, row_block=8)
        torch.cuda.synchronize()
        idx = band_frame_rows(row0, rows, step, 8).cuda()
        assert torch.equal(band.view(torch.int32), full[idx].view(torch.int32))
        for bad in [(0, 16, 24, 3), (0, 16, 4, 8), (8, 40, 48, 8), (0, 8, 1, 128)]:
            b0, brows, bstep, blk = bad
            with pytest.raises(vrt.VrtError):
                r.render_rows_async(cam, p, b0, brows, bstep, band.data_ptr(), stream=st, row_block=blk)


def test_c4_eight_way_split_at_full_size(built):
    """configs[4] at its full size: _TERRAIN 512^3, 3840x2160, (R,T) = (4,2), split over 8 ranks
    into 16-row block-cyclic bands (bench.py's and vrt_create(mask)'s split): every rank's band —
    through the timed path's launches (certified pass + deferred exact pass, automatic mode) and the
    in-lane exact path — equals its rows of the whole frame rendered by the exact STATS instance,
    bit for bit (the u_Alpha = 1 stored frame the bench times)."""
    n, w, h, R, T, world, block = 512, 3840, 2160, 4, 2, 8, 16
    with vrt.Renderer(0) as r:
        r.build_scene_device("terrain", n)
        cam = vrt.make_camera(w, h)
        full = band_frames(r, cam, R, T, 1.0, 0, h, 1, 1, 1, n_frames=1, counters=True)[0]
        for rank in range(world):
            row0, rows, step = block_band_spec(rank, world, h, block)
            idx = band_frame_rows(row0, rows, step, block).numpy()
            for mode in (1, 0):   # automatic deferred exact pass (the timed path), in-lane
                got = band_frames(r, cam, R, T, 1.0, row0, rows, step, block, mode, n_frames=1)[0]
                assert np.array_equal(got, full[idx]), (rank, mode)
