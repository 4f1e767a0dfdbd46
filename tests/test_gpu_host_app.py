"""The headless C++ host (examples/headless_app.cpp): AppScene's frame loop
driven through the C-ABI from C++. Its last filtered frame must equal the same frame sequence
rendered through the Python binding of the same library, byte for byte — per-frame u_Time, the
day/night clock, the temporal ping-pong, a history reset and textured mode included."""
import os
import subprocess

import numpy as np
import pytest

import voxelraytracer_amd as vrt

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(ROOT, "build", "bin", "vrt_headless")


def python_sequence(scene, n, w, h, frames, alpha, R, T, noise, frame_seconds, reset_at,
                    atlas=None, tile=128):
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene(scene, n), n)
        cam = vrt.make_camera(w, h)
        tod = 0.9 * 50.0
        out = None
        for f in range(frames):
            if f == reset_at:
                r.history_reset()
            p = vrt.default_params(R, T, time=float(f + 1), ray_noise=noise,
                                   sun_dir=vrt.sun_dir(np.float32(tod), 50.0))
            if atlas is not None:
                p = vrt.textured_params(p, atlas, tile)
            out, _ = r.render_frame(cam, p, alpha)
            if frame_seconds > 0:
                tod = np.float32(np.float32(tod) + np.float32(frame_seconds))
                while tod > 50.0:
                    tod = np.float32(tod - np.float32(50.0))
        return out


@pytest.mark.parametrize("textured", [False, True])
def test_headless_app_matches_python_binding(built, tmp_path, textured):
    assert os.path.exists(APP), "make app"
    scene, n, w, h, frames, alpha, noise, fs, reset = "terrain", 32, 96, 54, 4, 0.5, 0.02, 7.5, 2
    raw = tmp_path / "frame.rgba"
    ppm = tmp_path / "frame.ppm"
    cmd = [APP, "--scene", scene, "--n", str(n), "--size", f"{w}x{h}", "--frames", str(frames),
           "--alpha", str(alpha), "--ray-noise", str(noise), "--day-night", str(fs),
           "--reset-at", str(reset), "--bounces", "4", "2", "--raw", str(raw), "--ppm", str(ppm),
           "--quiet"]
    atlas = None
    if textured:
        atlas = vrt.make_atlas(64, 32, seed=3)
        atlas_file = tmp_path / "atlas.rgba"
        atlas_file.write_bytes(atlas.tobytes())
        cmd += ["--atlas-raw", str(atlas_file), "--atlas-size", "64", "--atlas-tile", "32"]
    subprocess.run(cmd, check=True, timeout=120)
    got = np.frombuffer(raw.read_bytes(), np.uint8).reshape(h, w, 4)
    ref = python_sequence(scene, n, w, h, frames, alpha, 4, 2, noise, fs, reset, atlas, 32)
    assert np.array_equal(got, ref)
    head = ppm.read_bytes()[:15]
    assert head.startswith(f"P6\n{w} {h}\n255\n".encode())
    img = np.frombuffer(ppm.read_bytes()[len(f"P6\n{w} {h}\n255\n"):], np.uint8).reshape(h, w, 3)
    assert np.array_equal(img, got[::-1, :, :3])   # screenshot: top row first
