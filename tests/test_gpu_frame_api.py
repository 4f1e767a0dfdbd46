"""GPU: the whole-frame entry points of the C-ABI (ABI v8) — the drop-in's fast path.

vrt_render_frame (main.cpp:323-393 as one call) now renders each device band as two interleaved
row parts on two context-owned streams with the fast (certified, uncounted) instance; timing
alone (vrt_stats.kernel_ms) no longer selects the exact-walk instance, counting does
(VRT_STATS_COUNTERS). Checked here:
  - frames are bit-identical to the exact instance's, over consecutive frames with alpha < 1;
  - a context over a device list splits the frame into 16-row block-cyclic bands (ABI v12;
    vrt_create_devices with a repeated ordinal rehearses a k-device split on one GPU; 121 rows:
    a short last block): identical frames, float frames and hit records;
  - vrt_render_frame_device assembles the same frame on the first device;
  - the C++ host (examples/headless_app.cpp) gets the bench's per-frame GPU time through the ABI.
The RCCL paths (ncclBroadcast of the volume, ncclGather of the bands) between distinct GPUs need
two of them; on the one-GPU test box they run with a one-rank communicator
(vrt_debug_collectives: the same calls, streams and assembly, no xGMI traffic)."""
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest
import torch

import voxelraytracer_amd as vrt

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(ROOT, "build", "bin", "vrt_headless")


def sequence(dev, scene, n, w, h, R, T, alphas, counters=False, **kw):
    with vrt.Renderer(dev) as r:
        r.upload_volume(vrt.build_scene(scene, n), n)
        cam = vrt.make_camera(w, h)
        out = []
        for i, a in enumerate(alphas):
            p = vrt.default_params(R, T, time=float(i + 1), **kw)
            f, st = r.render_frame(cam, p, a, counters=counters)
            out.append(f)
            if not counters:
                assert st["kernel_ms"] > 0 and st["pixels"] == 0
            else:
                assert st["pixels"] == w * h
        return out


CASES = [("refraction", 128, 480, 270, 4, 4, {}), ("glass_cube", 64, 320, 180, 1, 2, {}),
         ("terrain", 64, 256, 144, 4, 2, dict(ray_noise=0.02))]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_frame_fast_path_equals_exact_instance(built, case):
    scene, n, w, h, R, T, kw = case
    alphas = [1.0, 0.5, 0.5, 0.3]
    fast = sequence(0, scene, n, w, h, R, T, alphas, **kw)
    exact = sequence(0, scene, n, w, h, R, T, alphas, counters=True, **kw)
    for k, (a, b) in enumerate(zip(fast, exact)):
        assert np.array_equal(a, b), f"frame {k}"


@pytest.mark.parametrize("devs", [[0, 0], [0, 0, 0]], ids=["k2", "k3"])
def test_device_list_splits_frames_into_bands(built, devs):
    scene, n, w, h, R, T = "refraction", 64, 200, 121, 4, 4   # 121 rows: unequal bands
    alphas = [1.0, 0.5, 0.5]
    one = sequence(0, scene, n, w, h, R, T, alphas)
    many = sequence(devs, scene, n, w, h, R, T, alphas)
    for k, (a, b) in enumerate(zip(one, many)):
        assert np.array_equal(a, b), f"frame {k}"
    with vrt.Renderer(devs) as r, vrt.Renderer(0) as r1:
        assert r.device_count() == len(devs)
        vox = vrt.build_scene(scene, n)
        r.upload_volume(vox, n)
        r1.upload_volume(vox, n)
        cam = vrt.make_camera(w, h)
        p = vrt.default_params(R, T)
        for hits, counters in ((True, True), (False, False)):
            a, ha, sa = r.render(cam, p, want_hits=hits, counters=counters)
            b, hb, sb = r1.render(cam, p, want_hits=hits, counters=counters)
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
            if hits:
                assert np.array_equal(ha, hb)
            if counters:
                assert {k: v for k, v in sa.items() if k != "kernel_ms"} == \
                       {k: v for k, v in sb.items() if k != "kernel_ms"}


@pytest.mark.parametrize("devs", [0, [0, 0], "rccl1"], ids=["k1", "k2", "rccl1"])
def test_frame_device_output(built, devs):
    """vrt_render_frame_device hands out the frame on the first device (k1: the ring buffer it was
    rendered into; k2: the assembled bands; rccl1: one device through ncclBroadcast / ncclGather),
    identical to the synchronous frames; a frame stays valid for three more frames (the promise;
    the ring has eight slots)."""
    scene, n, w, h, R, T = "refraction", 128, 320, 181, 4, 4
    alphas = [1.0, 0.5, 0.5, 0.5, 0.7, 0.5, 0.4, 0.5]
    ref = sequence(0, scene, n, w, h, R, T, alphas)
    with vrt.Renderer(0 if devs == "rccl1" else devs) as r:
        if devs == "rccl1":
            r.debug_collectives()
        r.upload_volume(vrt.build_scene(scene, n), n)
        cam = vrt.make_camera(w, h)
        s = torch.cuda.Stream()
        ptrs = []
        ms = None
        for i, a in enumerate(alphas):
            s.wait_stream(torch.cuda.current_stream())
            ptr, t = r.render_frame_device(cam, vrt.default_params(R, T, time=float(i + 1)), a,
                                           s.cuda_stream, timing=(i == 1))
            ms = ms or (t["kernel_ms"] if t else None)
            ptrs.append(ptr)
            if i >= 3:   # frame i-3 is still valid after frame i
                torch.cuda.current_stream().wait_stream(s)
                for j in (i - 3, i):
                    got = np.empty((h, w, 4), np.uint8)
                    hipcopy(got, ptrs[j])
                    assert np.array_equal(got, ref[j]), f"frame {j} read after frame {i}"
        assert ms is not None and ms > 0
        assert len(set(ptrs)) == len(ptrs)   # ring of eight slots


@pytest.mark.parametrize("devs,null_stream", [(0, False), ([0, 0], False), (0, True), ([0, 0], True)],
                         ids=["k1", "k2", "k1-frame-stream", "k2-frame-stream"])
def test_device_frames_mixed_counted_and_alpha(built, devs, null_stream):
    """Device-output frames in flight (u_Alpha = 1: one launch per frame on rotating lanes) mixed
    with counted frames (the exact instance, one launch) and u_Alpha < 1 frames (two parts, each
    waiting for its history rows on another lane), plus a synchronous frame in between: every
    frame equals the synchronous sequence (a counted frame after uncounted device
    frames must be ordered after all of them)."""
    scene, n, w, h, R, T = "refraction", 128, 320, 181, 4, 4
    alphas = [1.0, 1.0, 0.5, 1.0, 1.0, 0.5, 0.6, 1.0, 1.0, 1.0, 0.5, 1.0]
    counted = {2, 4, 9}
    sync_at = {6}
    ref = sequence(0, scene, n, w, h, R, T, alphas)
    with vrt.Renderer(devs) as r:
        r.upload_volume(vrt.build_scene(scene, n), n)
        r.set_exact_pass(2)   # deferred exact passes at this small size too (automatic: in-lane)
        cam = vrt.make_camera(w, h)
        s = torch.cuda.Stream()
        for i, a in enumerate(alphas):
            p = vrt.default_params(R, T, time=float(i + 1))
            if i in sync_at:
                f, _ = r.render_frame(cam, p, a)
                assert np.array_equal(f, ref[i]), f"sync frame {i}"
                continue
            ptr, st = r.render_frame_device(cam, p, a, 0 if null_stream else s.cuda_stream,
                                            counters=i in counted)
            if i in counted:
                assert st["pixels"] == w * h
            got = np.empty((h, w, 4), np.uint8)
            if null_stream:   # consumed on the frame's own stream (vrt_frame_stream)
                fs = r.frame_stream()
                assert fs
                hipcopy_on(got, ptr, fs)
            else:
                torch.cuda.current_stream().wait_stream(s)
                hipcopy(got, ptr)
            assert np.array_equal(got, ref[i]), f"frame {i}"


@pytest.mark.parametrize("alpha", [0.5, 1.0])
def test_history_reset_keeps_held_frames(built, alpha):
    """Key F (vrt_history_reset, main.cpp:417-421) between device-output frames: the next frame
    filters against the last ray-traced frame, and the frames the caller still holds (valid until
    the fourth later call) keep their contents (the reset used to swap a held ring
    slot into the raw buffer, which the next frame overwrote)."""
    scene, n, w, h, R, T = "refraction", 128, 256, 144, 4, 4
    frames, reset_before = 7, 4
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene(scene, n), n)
        cam = vrt.make_camera(w, h)
        # reference through the band API: raw (quantised) and filtered frames, explicit history
        hist = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda")
        raw_prev = None
        refs = []
        cs = torch.cuda.current_stream().cuda_stream
        for i in range(frames):
            p = vrt.default_params(R, T, time=float(i + 1))
            prev = raw_prev if i == reset_before else hist
            cur = torch.zeros_like(hist)
            raw = torch.zeros_like(hist)
            r.render_temporal_rows_async(cam, p, alpha, 0, h, 1, prev.data_ptr(), cur.data_ptr(),
                                         raw.data_ptr(), stream=cs)
            torch.cuda.synchronize()
            refs.append(cur.cpu().numpy())
            hist, raw_prev = cur, raw
        s = torch.cuda.Stream()
        ptrs = []
        for i in range(frames):
            if i == reset_before:
                r.history_reset()
            ptr, _ = r.render_frame_device(cam, vrt.default_params(R, T, time=float(i + 1)), alpha,
                                           s.cuda_stream)
            ptrs.append(ptr)
            torch.cuda.current_stream().wait_stream(s)
            for j in range(max(0, i - 3), i + 1):   # every frame still held
                got = np.empty((h, w, 4), np.uint8)
                hipcopy(got, ptrs[j])
                assert np.array_equal(got, refs[j]), f"frame {j} read after frame {i}"


def hipcopy_on(dst: np.ndarray, ptr: int, stream_handle: int):
    """Device -> host copy of a raw device pointer enqueued on a raw HIP stream (the frame's own
    stream), then a wait for that stream."""
    class View:
        __cuda_array_interface__ = {"shape": dst.shape, "typestr": "|u1", "data": (ptr, False),
                                    "version": 3}

    ext = torch.cuda.ExternalStream(stream_handle)
    with torch.cuda.stream(ext):
        t = torch.as_tensor(View(), device="cuda").to("cpu", non_blocking=False)
    ext.synchronize()
    dst[...] = t.numpy()


def hipcopy(dst: np.ndarray, ptr: int):
    """Device -> host copy of a raw device pointer, viewed as a torch tensor through
    __cuda_array_interface__."""

    class View:
        __cuda_array_interface__ = {"shape": dst.shape, "typestr": "|u1", "data": (ptr, False),
                                    "version": 3}

    torch.cuda.synchronize()
    dst[...] = torch.as_tensor(View(), device="cuda").cpu().numpy()


def test_headless_app_gets_the_bench_frame_time(built, tmp_path):
    """vrt_headless (C++ over the C-ABI) at C3 in its display-path mode (--pipelined:
    vrt_render_frame_device with no caller stream, each frame consumed on the stream that produced
    it, no per-frame host sync): time per frame within 10 % of bench.py's per-frame GPU time of the
    same workload; the caller-stream form (--caller-stream) renders the same frames (both uncounted, certified, four
    frames in flight), the C++ host raising HIP's hardware-queue count itself as INTEGRATION.md
    asks (no GPU_MAX_HW_QUEUES in its environment). The synchronous loop
    (vrt_render_frame, which waits for each frame as the reference's blocking GL timer query did)
    reports each frame's own GPU time, which includes the frame's tail that consecutive frames
    hide; its frames are identical."""
    env = dict(os.environ)
    env.pop("GPU_MAX_HW_QUEUES", None)
    base = [APP, "--scene", "refraction", "--n", "128", "--size", "1920x1080", "--bounces", "4", "4",
            "--frames", "400", "--warmup", "200", "--quiet"]
    raw_p, raw_s, raw_c = tmp_path / "p.rgba", tmp_path / "s.rgba", tmp_path / "c.rgba"
    r = subprocess.run(base + ["--pipelined", "--raw", str(raw_p)], capture_output=True, text=True,
                       timeout=180, env=env)
    assert r.returncode == 0, r.stderr
    app_ms = float(re.search(r"mean ([0-9.]+) ms", r.stdout).group(1))
    rc = subprocess.run(base + ["--pipelined", "--caller-stream", "--raw", str(raw_c)], capture_output=True,
                        text=True, timeout=180, env=env)
    assert rc.returncode == 0, rc.stderr
    caller_ms = float(re.search(r"mean ([0-9.]+) ms", rc.stdout).group(1))
    assert raw_c.read_bytes() == raw_p.read_bytes()
    r2 = subprocess.run(base + ["--raw", str(raw_s)], capture_output=True, text=True, timeout=180, env=env)
    assert r2.returncode == 0, r2.stderr
    sync_ms = float(re.search(r"mean ([0-9.]+) ms", r2.stdout).group(1))
    assert raw_p.read_bytes() == raw_s.read_bytes()
    b = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "C3",
                        "--steps", "200", "--warmup", "200", "--cpu-seconds", "0", "--no-verify"],
                       capture_output=True, text=True, timeout=240)
    assert b.returncode == 0, b.stderr[-2000:]
    out = json.loads([l for l in b.stdout.splitlines() if l.startswith("{")][-1])
    bench_ms = out["roofline"]["kernel_ms"]
    print(f"vrt_headless pipelined {app_ms:.4f} ms/frame (frame streams), {caller_ms:.4f} ms/frame "
          f"(caller stream), synchronous {sync_ms:.4f} ms/frame, bench {bench_ms:.4f} ms/frame")
    assert app_ms <= 1.10 * bench_ms, (app_ms, bench_ms)


def test_launch_timing(built):
    """vrt_set_launch_timing / vrt_launch_timing: device start/end timestamps of async band
    launches (bench.py's launch_ms); launches past the requested count are not recorded."""
    n, w, h = 64, 320, 180
    with vrt.Renderer(0) as r:
        r.upload_volume(vrt.build_scene("refraction", n), n)
        cam = vrt.make_camera(w, h)
        p = vrt.default_params(4, 4)
        img = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        r.set_launch_timing(2)
        for _ in range(3):   # the third launch finds no free events
            r.render_rows_async(cam, p, 0, h, 1, img.data_ptr(), 0, 0, s)
        total, k = r.launch_timing()
        assert k == 2 and total > 0.0
        r.render_rows_async(cam, p, 0, h, 1, img.data_ptr(), 0, 0, s)   # events free again
        total2, k2 = r.launch_timing()
        assert k2 == 1 and total2 > 0.0
        r.set_launch_timing(0)
        r.render_rows_async(cam, p, 0, h, 1, img.data_ptr(), 0, 0, s)
        assert r.launch_timing() == (0.0, 0)
        torch.cuda.synchronize()
