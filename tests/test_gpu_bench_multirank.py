"""Rehearsal of bench.py's multi-rank path on a one-GPU box: torch.distributed.run with two ranks
sharing cuda:0 over gloo (RCCL needs one GPU per rank; the driver's 8-GPU run uses it). Checks the
JSON contract of rank 0's line for N = 2, strong and weak scaling (weak: the frame is 2 x 1080
rows), the per-frame gather of RGBA8 block-cyclic bands to rank 0 with frames in flight (the
default; over gloo here, the library's RCCL path in the driver's runs) or the bands kept on their
ranks with one gather after the timed region (--no-gather), and the max-over-ranks timing — the
code path the scaling runs take. A hang fails the test with every rank's Python stacks."""
import json
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("scaling,gather", [("weak", False), ("strong", False), ("weak", True),
                                            ("strong", True)])
def test_bench_two_ranks_json(built, scaling, gather):
    two_ranks(scaling, gather, ["--backend", "gloo", "--same-device"])


def test_bench_compositor_three_ranks(built):
    """--compositor 1 with three ranks on cuda:0 (gloo): rank 0 renders nothing, ranks 1 and 2
    split every frame (tiles.split_band_spec) and rank 0 assembles it; the gathered frames are
    checked against collect() and the roofline fields are renderer rank 1's."""
    out = two_ranks("strong", True, ["--backend", "gloo", "--same-device", "--compositor", "1"], n=3)
    assert out["gather"]["compositor"] is True and "rank 0 renders nothing" in out["config"]["parallelism"]
    assert out["roofline"]["rank"] == 1 and out["roofline"]["launch_ms"] > 0


def _device_count():
    import torch
    return torch.cuda.device_count()   # counts devices without initialising HIP in this process


@pytest.mark.skipif(_device_count() < 2, reason="RCCL needs one GPU per rank (the driver's multi-GPU node)")
@pytest.mark.parametrize("gather", [True, False])
def test_bench_two_ranks_rccl(built, gather):
    """The driver's N > 1 command itself on two GPUs: nccl backend (RCCL over xGMI), the library's
    per-lane communicators and ncclGather of RGB8 bands, rank 0's assembly checked bit for bit."""
    two_ranks("strong", gather, [])


@pytest.mark.skipif(_device_count() < 4, reason="RCCL needs one GPU per rank (the driver's multi-GPU node)")
def test_bench_four_ranks_rccl_compositor(built):
    """The driver's N = 4 command: RCCL, the compositor split by default (rank 0 assembles, ranks
    1-3 render), gathered frames checked bit for bit against collect()."""
    out = two_ranks("strong", True, [], n=4)
    assert out["gather"]["compositor"] is True and out["roofline"]["rank"] == 1


def two_ranks(scaling, gather, backend_args, n=2):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "6", "--warmup", "2",
           "--scaling", scaling, "--cpu-seconds", "0", "--watchdog-s", "100"] + backend_args
    cmd += [] if gather else ["--no-gather"]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    # own process group: a hung run is killed with its torchrun workers, after SIGUSR1 has made
    # every rank dump all its threads' Python stacks (bench.py registers faulthandler for it; the
    # ranks' --watchdog-s dump comes first) into the failure message
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=ROOT,
                         env=env, start_new_session=True)
    try:
        out_s, err_s = p.communicate(timeout=150)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGUSR1)
        time.sleep(3)
        os.killpg(p.pid, signal.SIGKILL)
        out_s, err_s = p.communicate()
        pytest.fail(f"{n}-rank bench did not finish in 150 s; rank stacks:\n" + err_s[-20000:])
    r = subprocess.CompletedProcess(cmd, p.returncode, out_s, err_s)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 prints exactly one JSON line
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline",
              "cpu_baseline", "latency", "gather"):
        assert k in out, k
    assert out["n_gpus"] == n and out["steps"] == 6 and out["scaling"] == scaling
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["config"]["frame"].startswith(f"1920x{1080 * n}" if scaling == "weak" else "1920x1080")
    assert out["roofline"]["kernel_ms_max_over_ranks"] >= out["roofline"]["kernel_ms"]
    assert out["cpu_baseline"] is None        # rank 0 at N=1 only
    assert out["verified"] is True
    assert out["latency"]["frame_latency_ms"] > 0
    rows = 1080 * n if scaling == "weak" else 1080
    assert out["verify"]["elements"] == rows * 1920 * 4   # every rank's band, summed: the frame
    if gather:   # every timed frame gathered and assembled on rank 0, checked against collect()
        assert out["collect"] is None and "every frame" in out["config"]["parallelism"]
        assert out["gather"]["per_frame"] is True and out["gather"]["render_only"]["value"] > 0
        assert out["verify"]["gathered_frame_mismatched_elements"] == 0
        # every rank enqueued each lane's gathers for the same frames (per-lane communicators)
        assert out["verify"]["gather_sequence_equal_all_ranks"] is True
        assert sum(out["verify"]["gathers_per_lane"]) > 0
        ro = out["gather"]["render_only"]
        assert ro["ms_per_step"] > 0 and ro["kernel_ms_max_over_ranks"] > 0
        bpp = 3 if (out["gather"]["wire"] or "").startswith("RGB8") else 4   # RCCL: RGB8 wire
        assert out["gather"]["bytes_to_rank0_per_frame"] == out["gather"]["band_rows_padded"] * 1920 * bpp * (n - 1)
    else:   # one gather of the last frame after the timed region
        assert out["collect"]["rows"] == rows and out["collect"]["bytes"] == rows * 1920 * 4
    return out
