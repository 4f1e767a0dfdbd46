"""GPU: the exact path the headline bench times, end to end (VERDICT r01 "Next round" #1).

bench.py renders C3 (_REFRACTION 128^3, 1920x1080, (R,T) = (4,4)) through FrameTiler: at alpha 1
four frames in flight on four lanes (streams + output buffers), at alpha 0.5 two interleaved row
parts on two HIP streams, written pitched into the frame and filtered in place; the heavy-first
tile order seeded by the frames before, certified walks. Here bench.py itself runs
that path and checks three consecutive frames after its timed region, each
  - bit for bit against the exact STATS instance (exact walks) rendering the same rows from a copy
    of the same history, and
  - within 1 LSB of the oracle's frame (oracle/vrt_oracle.c) through the oracle's RGB8 store and
    temporal filter (oracle_temporal) against the same history (colour is within 1e-4, which may
    straddle a rounding boundary of x*255; voxel.glsl:425-452, temporal.glsl:18, main.cpp:363-393).
alpha 0.5 makes every frame depend on the previous one, so a tile rendered twice or not at all
by the tile order, or a history read after its write, would show."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("alpha", [0.5, 1.0])
def test_bench_path_c3_three_frames(built, alpha):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "C3", "--steps", "20",
           "--warmup", "5", "--alpha", str(alpha), "--verify-frames", "3", "--cpu-seconds", "0",
           "--oracle-check", "--frame-events"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    v = out["verify"]
    assert v["frames"] == 3 and v["elements"] == 3 * 1920 * 1080 * 4
    assert v["verified"] and v["mismatched_elements"] == 0 and out["verified"]
    oc = out["oracle_check"]
    assert oc["frames"] == 3 and oc["ok"] and oc["max_lsb"] <= 1
    # per-frame completion events on each frame's own stream: one per frame, each after the
    # lanes' start and by the end of the timed frames
    ev = out["frame_events_ms"]
    assert len(ev) == 20 and all(0 < e <= 20 * out["roofline"]["kernel_ms"] * 1.01 + 1e-3 for e in ev)
    # alpha 1: frames independent, four in flight (lanes); else one lane of two parts in place
    par = out["config"]["parallelism"]
    if alpha == 1.0:
        assert out["roofline"]["lanes"] == 4 and "4 frames in flight" in par
    else:
        assert out["roofline"]["lanes"] == 1 and par.endswith("2 interleaved row parts per frame on 2 HIP streams")


@pytest.mark.parametrize("config", ["C1", "C2", "C4"])
def test_bench_path_other_configs(built, config):
    """The same end-to-end check for the other BASELINE GPU configs (full size): C1 (glass cube,
    exact primary walks: glass-heavy volume), C2 (terrain 128^3), C4 (terrain 512^3 at 3840x2160)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", config, "--steps", "10",
           "--warmup", "3", "--alpha", "0.5", "--verify-frames", "2", "--cpu-seconds", "0",
           "--oracle-check"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    v = out["verify"]
    w, h = out["config"]["width"], out["config"]["height"]
    assert v["frames"] == 2 and v["elements"] == 2 * w * h * 4
    assert v["verified"] and v["mismatched_elements"] == 0 and out["verified"]
    oc = out["oracle_check"]
    assert oc["frames"] == 2 and oc["ok"] and oc["max_lsb"] <= 1
