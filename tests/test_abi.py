"""The C-ABI boundary on the CPU: the library loads, exports every symbol include/vrt.h declares,
the ctypes mirror matches the header's layout, and the host harness (scene builders, camera, sun)
agrees with the oracle's independent restatement. No compute call touches a GPU here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import oracle
import voxelraytracer_amd as vrt
from voxelraytracer_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(ROOT, "include", "vrt.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\*\s]+?\b(vrt_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for name in ("vrt_create", "vrt_upload_volume", "vrt_render", "vrt_render_rows_async",
                 "vrt_destroy", "vrt_last_error"):
        assert name in fns


def test_library_exports_every_header_symbol(built):
    lib = C.CDLL(abi.LIB_PATH)
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert set(header_functions()) == set(abi.SIGNATURES), "ctypes mirror out of sync with vrt.h"


def test_struct_layouts():
    assert C.sizeof(abi.Camera) == 72
    assert C.sizeof(abi.Hit) == 16
    assert C.sizeof(abi.Params) == 64
    assert C.sizeof(abi.Stats) == 8 * abi.VRT_CNT_COUNT + 16
    assert np.dtype(abi.HIT_DTYPE).itemsize == C.sizeof(abi.Hit)


def test_abi_version(built):
    assert vrt.lib().vrt_abi_version() == 15


@pytest.mark.parametrize("scene", [0, 1, 2])
@pytest.mark.parametrize("n", [8, 16, 32, 64, 128, 256])
def test_scene_builders_match_oracle(built, scene, n):
    a = vrt.build_scene(scene, n)
    b = oracle.build_scene(scene, n)
    assert np.array_equal(a, b)


def test_terrain_noise_matches_oracle(built):
    for n in (16, 32, 128, 512):
        assert np.array_equal(vrt.terrain_noise(n), oracle.terrain_noise(n))


def test_invalid_scene_rejected(built):
    with pytest.raises(vrt.VrtError):
        vrt.build_scene(7, 16)


def test_camera_looks_into_the_volume(built):
    cam = vrt.make_camera(64, 36)
    m = np.array(cam.inv_pv, np.float64).reshape(4, 4).T   # row-major view of column-major data
    near = m @ np.array([0, 0, -1, 1.0])
    near = near[:3] / near[3]
    # the near-plane centre sits 0.01 in front of the camera at main.cpp:171's position
    assert np.linalg.norm(near - np.array(vrt.DEFAULT_CAM_POS)) == pytest.approx(0.01, rel=1e-3)


def test_sun_direction_make_day(built):
    s = np.array(vrt.sun_dir(0.9 * 50.0, 50.0))
    assert abs(np.linalg.norm(s) - 1) < 1e-6
    assert s[1] > 0.7    # daytime: the sky term max(u_SunDir.y, 0) is on (voxel.glsl:391)
    assert s[2] > 0


def test_create_without_gpu_fails_loudly(built):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(vrt.VrtError):
        vrt.Renderer(0)


@pytest.mark.parametrize("height,k,parts", [(1080, 1, 2), (1080, 2, 2), (1080, 8, 2), (2160, 8, 2),
                                            (7, 3, 2), (5, 8, 2), (1, 1, 2), (100, 3, 1)])
def test_band_plan_covers_every_row_once(built, height, k, parts):
    """vrt_band_plan (the whole-frame split of vrt_render / vrt_render_frame over k devices and
    their interleaved parts): every frame row is rendered by exactly one part, into band row r of
    band j with frame row = j + r*k, and every band fits the largest band's rows."""
    plan, cap = vrt.band_plan(height, k, parts)
    assert cap == -(-height // k)
    seen = np.zeros(height, np.int32)
    for (j, p), (row0, rows, step, brow0) in plan.items():
        assert step == k * parts and brow0 == p
        for i in range(rows):
            frame_row = row0 + i * step
            band_row = brow0 + i * parts
            assert band_row < cap
            assert frame_row == j + band_row * k
            seen[frame_row] += 1
    assert np.all(seen == 1)


def test_band_plan_composes_the_oracle_frame(built):
    """The library's placement of multi-device band parts (vrt_band_plan + the per-device strided
    copies into host rows) reproduces the whole frame, with the oracle as the band renderer."""
    n, w, h, k, parts = 16, 40, 27, 3, 2
    vox = vrt.build_scene("refraction", n)
    cam = vrt.make_camera(w, h)
    p = vrt.default_params(4, 4)
    full, _, _ = oracle.render(cam, vox, n, p)
    plan, cap = vrt.band_plan(h, k, parts)
    bands = np.full((k, cap, w, 4), np.nan, np.float32)
    for (j, q), (row0, rows, step, brow0) in plan.items():
        if rows:
            part, _, _ = oracle.render(cam, vox, n, p, row0=row0, rows=rows, row_step=step)
            bands[j, brow0::parts][:rows] = part
    frame = np.full((h, w, 4), np.nan, np.float32)
    for j in range(k):
        hb = len(range(j, h, k))
        frame[j::k] = bands[j, :hb]   # hipMemcpy2D: dst pitch k*W, src pitch W
    assert np.array_equal(frame.view(np.uint32), full.view(np.uint32))


def _memcpy2d(dst, dst_off, dst_pitch, src, src_pitch, width, rows):
    for r in range(rows):   # hipMemcpy2D semantics, byte for byte
        d = dst_off + r * dst_pitch
        assert 0 <= d and d + width <= dst.size, "copy out of the frame"
        assert r * src_pitch + width <= src.size, "copy out of the band"
        dst[d:d + width] = src[r * src_pitch:r * src_pitch + width]


@pytest.mark.parametrize("width,height,k,elem", [(40, 27, 4, 4), (1920, 1081, 8, 4), (33, 7, 3, 16),
                                                 (5, 5, 8, 16), (64, 1080, 7, 16), (3, 1, 1, 4)])
def test_band_copy_plan_assembles_unequal_bands(built, width, height, k, elem):
    """The copies the library issues to assemble a multi-device frame (pinned host staging of
    vrt_render / vrt_render_frame, and the device-frame gather) place every band's packed rows at
    their frame rows, each frame byte written once, when height % k != 0 leaves bands of unequal
    height (and some empty when k > height): applied here with hipMemcpy2D's semantics."""
    plan = vrt.band_copy_plan(width, height, k, elem)
    row = width * elem
    frame = np.zeros(height * row, np.uint8)
    written = np.zeros(height * row, np.int32)
    for j, (dst_off, dst_pitch, src_pitch, wbytes, rows) in enumerate(plan):
        assert rows == len(range(j, height, k)) and wbytes == row and src_pitch == row
        # band j: packed rows, each filled with a pattern naming its frame row and band
        band = np.zeros(max(rows, 1) * row, np.uint8)
        for r in range(rows):
            band[r * row:(r + 1) * row] = (j + r * k) * 7 + j + 1 & 0xFF
        _memcpy2d(frame, dst_off, dst_pitch, band, src_pitch, wbytes, rows)
        ones = np.zeros_like(written)
        _memcpy2d(ones, dst_off, dst_pitch, np.ones(max(rows, 1) * row, np.int32), src_pitch, wbytes, rows)
        written += ones
    assert np.all(written == 1)
    for fr in range(height):
        j = fr % k
        assert np.all(frame[fr * row:(fr + 1) * row] == (fr * 7 + j + 1) & 0xFF)


@pytest.mark.parametrize("height,k,block", [(1080, 2, 16), (1080, 8, 16), (2160, 8, 16), (1081, 3, 16),
                                            (7, 3, 4), (5, 8, 16), (100, 1, 16), (4000, 7, 64)])
def test_block_band_plan_covers_every_row_once(built, height, k, block):
    """vrt_block_band_plan (ABI v12: the whole-frame split over k > 1 devices): every frame row is
    rendered by exactly one band, band row i = frame row row0 + (i // B) * step + i % B, the
    largest band is band 0's, and the plan equals tiles.block_band_spec (bench.py's split)."""
    from voxelraytracer_amd.tiles import block_band_spec

    plan, cap = vrt.block_band_plan(height, k, block)
    seen = np.zeros(height, np.int32)
    for j, (row0, rows, step) in enumerate(plan):
        assert (row0, rows, step) == block_band_spec(j, k, height, block)
        assert rows <= cap
        for i in range(rows):
            seen[row0 + (i // block) * step + i % block] += 1
    assert np.all(seen == 1)
    assert cap == max(r for _, r, _ in plan)


def test_frame_row_block(built):
    assert vrt.frame_row_block(1) == 1 and vrt.frame_row_block(2) == 16 and vrt.frame_row_block(8) == 16


@pytest.mark.parametrize("width,height,k,block,elem", [(40, 27, 4, 4, 4), (1920, 1081, 8, 16, 4),
                                                       (33, 7, 3, 2, 16), (5, 5, 8, 16, 16),
                                                       (64, 1080, 7, 16, 16), (3, 1, 1, 16, 4),
                                                       (3840, 2160, 8, 16, 4)])
def test_block_copy_plan_assembles_unequal_bands(built, width, height, k, block, elem):
    """The copies the library issues to assemble a multi-device frame from block-cyclic bands
    (ABI v12: staging of vrt_render / vrt_render_frame, the repeated-device gather): every frame
    byte written once, from the band row that renders it, with hipMemcpy2D's semantics."""
    plan, cap = vrt.block_band_plan(height, k, block)
    copies = vrt.block_copy_plan(width, height, k, block, elem)
    row = width * elem
    frame = np.zeros(height * row, np.uint8)
    written = np.zeros(height * row, np.int32)
    bands = []
    for j, (row0, rows, step) in enumerate(plan):
        band = np.zeros(max(cap, 1) * row, np.uint8)
        for i in range(rows):   # band row i holds a pattern naming its frame row
            fr = row0 + (i // block) * step + i % block
            band[i * row:(i + 1) * row] = (fr * 7 + 3) & 0xFF
        bands.append(band)
    for j, dst_off, dst_pitch, src_off, src_pitch, wbytes, rows in copies:
        _memcpy2d(frame, dst_off, dst_pitch, bands[j][src_off:], src_pitch, wbytes, rows)
        ones = np.zeros_like(written)
        _memcpy2d(ones, dst_off, dst_pitch, np.ones(bands[j].size - src_off, np.int32), src_pitch, wbytes, rows)
        written += ones
    assert np.all(written == 1)
    for fr in range(height):
        assert np.all(frame[fr * row:(fr + 1) * row] == (fr * 7 + 3) & 0xFF)


def test_block_bands_compose_the_oracle_frame(built):
    """The library's k-device split (block-cyclic bands, one launch per band) with the oracle as the
    band renderer and the library's copy plan as the assembly reproduces the whole frame."""
    n, w, h, k = 16, 40, 53, 3
    block = vrt.frame_row_block(k)
    vox = vrt.build_scene("refraction", n)
    cam = vrt.make_camera(w, h)
    p = vrt.default_params(4, 4)
    full, _, _ = oracle.render(cam, vox, n, p)
    plan, cap = vrt.block_band_plan(h, k, block)
    bands = []
    for row0, rows, step in plan:
        b = np.full((cap, w, 4), np.nan, np.float32)
        for i in range(rows):
            fr = row0 + (i // block) * step + i % block
            b[i] = oracle.render(cam, vox, n, p, row0=fr, rows=1)[0][0]
        bands.append(b.reshape(-1).view(np.uint8))
    frame = np.zeros(h * w * 16, np.uint8)
    for j, dst_off, dst_pitch, src_off, src_pitch, wbytes, rows in vrt.block_copy_plan(w, h, k, block, 16):
        _memcpy2d(frame, dst_off, dst_pitch, bands[j][src_off:], src_pitch, wbytes, rows)
    assert np.array_equal(frame.view(np.uint32), full.reshape(-1).view(np.uint8).view(np.uint32))


def test_headless_app_builds_and_parses(built):
    """examples/headless_app.cpp links against the C-ABI (make app); --help needs no GPU."""
    import subprocess

    app = os.path.join(ROOT, "build", "bin", "vrt_headless")
    assert os.path.exists(app)
    r = subprocess.run([app, "--help"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 2 and "--scene" in r.stdout
    r = subprocess.run([app, "--bogus"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 2
