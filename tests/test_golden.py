"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py from the cross-checked
CPU oracle): the oracle and the scene builders reproduce them exactly on the CPU; the HIP kernel
reproduces them on the GPU (hit records bit-exact, colour within 1e-4)."""
import glob
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
import voxelraytracer_amd as vrt
from voxelraytracer_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
FILES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


def load(path):
    z = np.load(path, allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    cam = abi.Camera()
    cam.inv_pv = (abi.C.c_float * 16)(*z["inv_pv"].tolist())
    cam.width, cam.height = meta["width"], meta["height"]
    p = vrt.default_params(meta["params"]["max_reflections"], meta["params"]["max_transparencies"])
    for k, v in meta["params"].items():
        if k == "sun_dir":
            p.sun_dir = (abi.C.c_float * 3)(*v)
        else:
            setattr(p, k, v)
    if "atlas" in z.files and z["atlas"].size:
        p = vrt.textured_params(p, z["atlas"], meta["params"]["atlas_texture_size"])
    vox = vrt.build_scene(meta["scene"], meta["n"], meta["seed"])
    return z, meta, cam, p, vox


def test_reference_atlas_fixture():
    """tests/golden/atlas/atlas_ref128.npz holds the reference's decoded textures
    (main.cpp:187-193): 256x256 RGBA8, opaque stone/dirt/grass, glass alpha exactly {0, 255}."""
    z = np.load(os.path.join(HERE, "golden", "atlas", "atlas_ref128.npz"), allow_pickle=False)
    a = z["atlas"]
    meta = json.loads(str(z["meta"]))
    assert a.shape == (256, 256, 4) and a.dtype == np.uint8
    assert set(meta["png_sha256"]) == {f"{k}128.png" for k in vrt.ATLAS_SLOTS}
    for name, (tx, ty) in vrt.ATLAS_SLOTS.items():
        rs, cs = vrt.atlas_slot_rows(256, 128, tx, ty)
        alpha = np.unique(a[rs, cs, 3])
        if name == "glass":
            assert alpha.tolist() == [0, 255]
        else:
            assert alpha.tolist() == [255]


def test_fixtures_present():
    assert len(FILES) >= 6


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[:-4] for f in FILES])
def test_oracle_reproduces_golden(built, path):
    z, meta, cam, p, vox = load(path)
    assert hashlib.sha256(vox.tobytes()).hexdigest() == meta["volume_sha256"]
    rgba, hits, cnt = oracle.render(cam, vox, meta["n"], p, threads=4)
    assert np.array_equal(rgba.view(np.uint32), z["rgba"].view(np.uint32))
    assert np.array_equal(hits["voxel_index"], z["voxel_index"])
    assert np.array_equal(hits["ray_length"].view(np.uint32), z["ray_length_bits"])
    assert np.array_equal(hits["steps"], z["steps"])
    assert np.array_equal(hits["flags"], z["flags"])
    assert cnt == meta["counters"]


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[:-4] for f in FILES])
def test_gpu_reproduces_golden(built, path):
    z, meta, cam, p, vox = load(path)
    with vrt.Renderer(0) as r:
        r.upload_volume(vox, meta["n"])
        rgba, hits, st = r.render(cam, p)
    assert np.array_equal(hits["voxel_index"], z["voxel_index"])
    assert np.array_equal(hits["ray_length"].view(np.uint32), z["ray_length_bits"])
    assert np.array_equal(hits["steps"], z["steps"])
    assert np.array_equal(hits["flags"], z["flags"])
    for k, v in meta["counters"].items():
        assert st[k] == v, k
    d = np.abs(np.clip(rgba[..., :3], 0, 1) - np.clip(z["rgba"][..., :3], 0, 1)).max()
    assert d <= 1e-4, d
