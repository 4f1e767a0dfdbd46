"""FrameTiler on the GPU with the real HIP kernel: two ranks (processes) sharing cuda:0 over the
gloo backend with CUDA tensors (RCCL needs one GPU per rank; the driver's 8-GPU run uses it).
Exercises the CUDA-only parts of the multi-GPU path — uint8 RGBA8 block-cyclic bands, the
temporal history carried in the previous lane's band buffer, the per-frame gather and rank 0's
re-interleave on the frame's lane stream — and checks the assembled frames against a
single-process render of the same frames, bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, W, H, FRAMES, ALPHA = 32, 128, 72, 4, 0.5


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def frame_params(vrt, t):
    return vrt.default_params(4, 2, time=float(t + 1), ray_noise=0.03)


def worker(rank, world, port, q, lanes, row_block):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import voxelraytracer_amd as vrt
    from voxelraytracer_amd.tiles import FrameTiler, broadcast_volume, row_pitch

    dev = torch.device("cuda", 0)
    vox = torch.from_numpy(vrt.build_scene("terrain", N)).to(dev) if rank == 0 else \
        torch.zeros(N ** 3, dtype=torch.uint8, device=dev)
    broadcast_volume(vox)
    ren = vrt.Renderer(0)
    ren.upload_volume_device(vox.data_ptr(), N, torch.cuda.current_stream().cuda_stream)
    cam = vrt.make_camera(W, H)
    state = {"t": 0}

    def render_band(row0, rows, step, out, prev, row_block=1):
        ren.render_temporal_rows_async(cam, frame_params(vrt, state["t"]), ALPHA, row0,
                                       rows, step, prev.data_ptr(), out.data_ptr(),
                                       stream=torch.cuda.current_stream().cuda_stream,
                                       pitch=row_pitch(out), row_block=row_block)
        state["t"] += 1

    tiler = FrameTiler(W, H, render_band, dev, dtype=torch.uint8, lanes=lanes, row_block=row_block)
    got = []
    for _ in range(FRAMES):
        f = tiler.frame()
        if f is not None:
            torch.cuda.synchronize()
            got.append(f.cpu().numpy())
    f = tiler.finish()
    torch.cuda.synchronize()
    if f is not None:
        assert np.array_equal(f.cpu().numpy(), got[-1])
    if rank == 0:
        q.put(got)
    dist.barrier()
    ren.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("lanes,row_block", [(1, 1), (3, 16), (2, 8)])
def test_two_ranks_on_one_gpu_match_single_process(built, lanes, row_block):
    import voxelraytracer_amd as vrt

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q, lanes, row_block)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(got) == FRAMES
    with vrt.Renderer(0) as ren:
        ren.upload_volume(vrt.build_scene("terrain", N), N)
        cam = vrt.make_camera(W, H)
        hist = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        for t in range(FRAMES):
            ren.render_temporal_rows_async(cam, frame_params(vrt, t), ALPHA, 0, H, 1,
                                           hist.data_ptr(), hist.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(got[t], hist.cpu().numpy()), t


def test_single_rank_two_streams_match(built):
    """One rank, two interleaved parts on two HIP streams (the bench default): each part renders
    into its rows of the frame through the row pitch and filters them in place; each frame
    returned by the tiler equals the single-stream filtered frame."""
    import voxelraytracer_amd as vrt
    from voxelraytracer_amd.tiles import FrameTiler, row_pitch

    with vrt.Renderer(0) as ren:
        ren.upload_volume(vrt.build_scene("terrain", N), N)
        cam = vrt.make_camera(W, H)
        state = {"t": 0}

        def render_band(row0, rows, step, out, prev):
            ren.render_temporal_rows_async(cam, frame_params(vrt, state["t"] // 2), ALPHA, row0,
                                           rows, step, prev.data_ptr(), out.data_ptr(),
                                           stream=torch.cuda.current_stream().cuda_stream,
                                           pitch=row_pitch(out))
            state["t"] += 1

        tiler = FrameTiler(W, H, render_band, torch.device("cuda", 0), dtype=torch.uint8, parts=2)
        hist = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        for t in range(FRAMES):
            f = tiler.frame()
            torch.cuda.synchronize()
            got = f.cpu().numpy()
            ren.render_temporal_rows_async(cam, frame_params(vrt, t), ALPHA, 0, H, 1,
                                           hist.data_ptr(), hist.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(got, hist.cpu().numpy()), t
        tiler.finish()
