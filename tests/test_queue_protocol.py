"""CPU: the fused frame's queue protocol (frame_kernel / drain_kernel in vrt_render.hip) under a
threaded stress model (tests/queue_model.cpp): every queued pixel claimed and rendered exactly
once (owned full batches, class drains, the drain kernel), across 200 random schedules, with and
without a heavy-first pass."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_queue_protocol_model(tmp_path):
    exe = tmp_path / "queue_model"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-o", str(exe),
                           os.path.join(ROOT, "tests", "queue_model.cpp")])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
