"""Multi-rank framebuffer tiling (voxelraytracer_amd/tiles.py) on CPU with the gloo backend.

Each rank renders its cyclic row band with the CPU oracle standing in for the HIP kernel (the
same render_band contract bench.py feeds with vrt_render_rows_async), rank 0 gathers and
re-interleaves; the assembled frames of a pipelined sequence must equal single-process oracle
frames bit for bit. Also checks the volume broadcast."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, n, w, h, frames, q, mode="f32", alpha=0.5, parts=1, gather=True,
           lanes=1, row_block=1, compositor=False):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    import voxelraytracer_amd as vrt
    from voxelraytracer_amd.tiles import FrameTiler, band_frame_rows, broadcast_volume

    vox = torch.from_numpy(vrt.build_scene("glass_cube", n)) if rank == 0 else \
        torch.zeros(n ** 3, dtype=torch.uint8)
    broadcast_volume(vox)
    vox_np = vox.numpy()
    cam = vrt.make_camera(w, h)
    params = [vrt.default_params(1, 2, time=float(t + 1), ray_noise=0.05) for t in range(frames)]
    state = {"i": 0}

    def render_band(row0, rows, step, out, prev, row_block=1):
        if row_block > 1:   # block-cyclic band: the band's frame rows of a whole oracle frame
            full, _, _ = oracle.render(cam, vox_np, n, params[state["i"] // parts], threads=1)
            rgba = full[band_frame_rows(row0, rows, step, row_block).numpy()]
        else:
            rgba, _, _ = oracle.render(cam, vox_np, n, params[state["i"] // parts], row0=row0,
                                       rows=rows, row_step=step, threads=1)
        if mode == "rgba8":   # the fused temporal filter + RGB8 store, band-local history
            _, cur = oracle.temporal(rgba, prev.numpy().copy(), alpha)
            out.copy_(torch.from_numpy(cur))
        else:
            out.copy_(torch.from_numpy(rgba))
        state["i"] += 1

    tiler = FrameTiler(w, h, render_band, torch.device("cpu"),
                       dtype=torch.uint8 if mode == "rgba8" else torch.float32, parts=parts,
                       gather=gather, lanes=lanes, row_block=row_block, compositor=compositor)
    got = []
    for _ in range(frames):
        f = tiler.frame()
        if gather:   # rank 0: the frame just rendered, gathered and assembled
            assert (f is not None) == (rank == 0)
            if f is not None:
                got.append(f.clone().numpy())
        else:   # bands stay on their ranks; gather each frame here only to check it
            tiler.finish()
            full = tiler.collect()
            if rank == 0:
                got.append(full.clone().numpy())
    f = tiler.finish()
    if gather and rank == 0:
        assert np.array_equal(f.numpy(), got[-1])
    if gather:   # every rank enqueued the same frames' exchanges on every lane (bench.py checks it)
        xl = torch.tensor(tiler.exchange_log(), dtype=torch.int64)
        lo, hi = xl.clone(), xl.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        assert torch.equal(lo, hi) and int(xl[0::2].sum()) == frames, xl.tolist()
    if rank == 0:
        q.put((got, bytes(vox_np)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,lanes,row_block", [(2, 1, 1), (3, 1, 1), (2, 3, 1), (3, 2, 4), (2, 4, 8)])
def test_tiled_frames_match_single_process(built, world, lanes, row_block):
    """The per-frame gather (bench.py's multi-rank default): cyclic or block-cyclic bands (ragged:
    18 rows over 3 ranks in blocks of 4), frames in flight on several lanes; rank 0's assembled
    frames equal single-process oracle frames bit for bit."""
    import oracle
    import voxelraytracer_amd as vrt

    n, w, h, frames = 16, 24, 18, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, w, h, frames, q, "f32", 0.5,
                                              1, True, lanes, row_block)) for r in range(world)]
    for p in procs:
        p.start()
    got, vox_bytes = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    vox = vrt.build_scene("glass_cube", n)
    assert vox_bytes == vox.tobytes()   # broadcast replicated the volume
    cam = vrt.make_camera(w, h)
    assert len(got) == frames
    for t in range(frames):
        ref, _, _ = oracle.render(cam, vox, n, vrt.default_params(1, 2, time=float(t + 1),
                                                                  ray_noise=0.05))
        assert np.array_equal(got[t].view(np.uint32), ref.view(np.uint32)), t


def test_band_spec_and_assembly():
    from voxelraytracer_amd.tiles import assemble_cyclic, band_spec

    assert band_spec(1, 4, 1080) == (1, 270, 4)
    with pytest.raises(ValueError):
        band_spec(0, 7, 1080)
    frame = torch.arange(12 * 2 * 1, dtype=torch.float32).reshape(12, 2, 1)
    bands = torch.stack([frame[r::3] for r in range(3)])
    assert torch.equal(assemble_cyclic(bands), frame)


@pytest.mark.parametrize("lanes,row_block", [(1, 1), (2, 4), (3, 2)])
def test_tiled_temporal_rgba8_frames(built, lanes, row_block):
    """RGBA8 bands with the temporal filter, gathered every frame (dependent lanes at alpha 0.5):
    each rank's history is its own band of the previous frame, so the assembled sequence equals
    the single-process filtered sequence bit for bit."""
    import oracle
    import voxelraytracer_amd as vrt

    n, w, h, frames, world, alpha = 16, 20, 12, 4, 2, 0.5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, w, h, frames, q, "rgba8", alpha,
                                              1, True, lanes, row_block)) for r in range(world)]
    for p in procs:
        p.start()
    got, _ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    vox = vrt.build_scene("glass_cube", n)
    cam = vrt.make_camera(w, h)
    hist = np.zeros((h, w, 4), np.uint8)
    assert len(got) == frames
    for t in range(frames):
        rgba, _, _ = oracle.render(cam, vox, n, vrt.default_params(1, 2, time=float(t + 1),
                                                                   ray_noise=0.05))
        _, hist = oracle.temporal(rgba, hist, alpha)
        assert np.array_equal(got[t], hist), t


@pytest.mark.parametrize("parts", [2, 3])
def test_single_rank_parts(built, parts):
    """One rank, several interleaved parts (the bench's tail-hiding split): the frame returned
    each step equals the single-part filtered sequence."""
    import oracle
    import voxelraytracer_amd as vrt
    from voxelraytracer_amd.tiles import FrameTiler

    n, w, h, frames, alpha = 16, 20, 12, 3, 0.5
    vox = vrt.build_scene("glass_cube", n)
    cam = vrt.make_camera(w, h)
    state = {"i": 0}

    def render_band(row0, rows, step, out, prev):
        p = vrt.default_params(1, 2, time=float(state["i"] // parts + 1), ray_noise=0.05)
        rgba, _, _ = oracle.render(cam, vox, n, p, row0=row0, rows=rows, row_step=step)
        _, cur = oracle.temporal(rgba, prev.numpy().copy(), alpha)
        out.copy_(torch.from_numpy(cur))
        state["i"] += 1

    tiler = FrameTiler(w, h, render_band, torch.device("cpu"), dtype=torch.uint8, parts=parts)
    hist = np.zeros((h, w, 4), np.uint8)
    for t in range(frames):
        got = tiler.frame().numpy().copy()
        rgba, _, _ = oracle.render(cam, vox, n, vrt.default_params(1, 2, time=float(t + 1),
                                                                   ray_noise=0.05))
        _, hist = oracle.temporal(rgba, hist, alpha)
        assert np.array_equal(got, hist), t
    assert np.array_equal(tiler.finish().numpy(), hist)


def test_part_spec_and_assembly():
    from voxelraytracer_amd.tiles import assemble_parts, part_spec

    assert part_spec(1, 4, 1, 2, 1080) == (5, 135, 8)
    with pytest.raises(ValueError):
        part_spec(0, 8, 0, 2, 1080)
    frame = torch.arange(12 * 2, dtype=torch.float32).reshape(12, 2, 1)
    world, parts = 2, 3
    g = torch.stack([torch.stack([frame[s * world + r::world * parts] for s in range(parts)])
                     for r in range(world)])
    assert torch.equal(assemble_parts(g), frame)


@pytest.mark.parametrize("world,parts", [(2, 1), (2, 2), (3, 2)])
def test_distributed_bands_without_per_frame_gather(built, world, parts):
    """gather=False (bench.py's multi-rank default): every rank renders and filters its own band
    in place with no exchange; collect() assembles the frame on rank 0 — the RGBA8 temporal
    sequence equals the single-process one bit for bit."""
    import oracle
    import voxelraytracer_amd as vrt

    n, w, h, frames, alpha = 16, 20, 12, 3, 0.5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, w, h, frames, q, "rgba8", alpha,
                                              parts, False)) for r in range(world)]
    for p in procs:
        p.start()
    got, _ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    vox = vrt.build_scene("glass_cube", n)
    cam = vrt.make_camera(w, h)
    hist = np.zeros((h, w, 4), np.uint8)
    assert len(got) == frames
    for t in range(frames):
        rgba, _, _ = oracle.render(cam, vox, n, vrt.default_params(1, 2, time=float(t + 1),
                                                                   ray_noise=0.05))
        _, hist = oracle.temporal(rgba, hist, alpha)
        assert np.array_equal(got[t], hist), t


@pytest.mark.parametrize("lanes,parts,independent", [(3, 1, False), (2, 2, False), (4, 1, True)])
def test_single_rank_lanes(built, lanes, parts, independent):
    """Frames in flight (bench.py's default at alpha 1): frame k renders into lane k % L's buffer
    and reads its history from the previous lane's. Dependent lanes (alpha 0.5) must give the
    single-buffer filtered sequence; independent lanes (alpha 1: the history is not read) the
    quantised frames. Each returned band is the frame, and stays valid for L - 1 more frames."""
    import oracle
    import voxelraytracer_amd as vrt
    from voxelraytracer_amd.tiles import FrameTiler

    n, w, h, frames = 16, 20, 12, 6
    alpha = 1.0 if independent else 0.5
    vox = vrt.build_scene("glass_cube", n)
    cam = vrt.make_camera(w, h)
    state = {"i": 0}

    def render_band(row0, rows, step, out, prev):
        p = vrt.default_params(1, 2, time=float(state["i"] // parts + 1), ray_noise=0.05)
        rgba, _, _ = oracle.render(cam, vox, n, p, row0=row0, rows=rows, row_step=step)
        old = np.full_like(prev.numpy(), 77) if independent else prev.numpy().copy()
        _, cur = oracle.temporal(rgba, old, alpha)   # alpha 1: independent of the history
        out.copy_(torch.from_numpy(cur))
        state["i"] += 1

    tiler = FrameTiler(w, h, render_band, torch.device("cpu"), dtype=torch.uint8, parts=parts,
                       lanes=lanes, independent=independent)
    hist = np.zeros((h, w, 4), np.uint8)
    kept = []
    for t in range(frames):
        f = tiler.frame()
        kept.append((f, tiler.last()))
        rgba, _, _ = oracle.render(cam, vox, n, vrt.default_params(1, 2, time=float(t + 1),
                                                                   ray_noise=0.05))
        _, hist = oracle.temporal(rgba, hist, alpha)
        assert f is tiler.bufs[t % lanes] and kept[-1][1] is f
        assert np.array_equal(f.numpy(), hist), t
    assert np.array_equal(tiler.finish().numpy(), hist)


def test_lanes_need_kept_bands():
    from voxelraytracer_amd.tiles import FrameTiler

    with pytest.raises(ValueError):
        FrameTiler(8, 4, lambda *a: None, torch.device("cpu"), lanes=0)


@pytest.mark.parametrize("world,lanes", [(2, 2), (2, 3)])
def test_distributed_lanes(built, world, lanes):
    """Several ranks keeping their bands, each with frames in flight (bench.py's multi-GPU
    default at alpha 1, here with dependent lanes at alpha 0.5): the collected frames equal the
    single-process sequence."""
    import oracle
    import voxelraytracer_amd as vrt

    n, w, h, frames, alpha = 16, 20, 12, 4, 0.5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, w, h, frames, q, "rgba8", alpha,
                                              1, False, lanes)) for r in range(world)]
    for p in procs:
        p.start()
    got, _ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    vox = vrt.build_scene("glass_cube", n)
    cam = vrt.make_camera(w, h)
    hist = np.zeros((h, w, 4), np.uint8)
    assert len(got) == frames
    for t in range(frames):
        rgba, _, _ = oracle.render(cam, vox, n, vrt.default_params(1, 2, time=float(t + 1),
                                                                   ray_noise=0.05))
        _, hist = oracle.temporal(rgba, hist, alpha)
        assert np.array_equal(got[t], hist), t


def test_block_band_spec_covers_the_frame():
    """Block-cyclic bands (ABI v11 row_block): every frame row exactly once, bands within one
    block of each other, block 1 = the cyclic band, ragged heights and more ranks than blocks."""
    from voxelraytracer_amd.tiles import band_frame_rows, band_spec, block_band_spec

    assert block_band_spec(1, 4, 1080, 1) == band_spec(1, 4, 1080)
    assert block_band_spec(0, 8, 1080, 8) == (0, 136, 64)   # 135 blocks: ranks 0-6 get 17
    assert block_band_spec(7, 8, 1080, 8) == (56, 128, 64)
    for h, world, b in [(1080, 8, 8), (2160, 8, 8), (21, 3, 4), (12, 2, 8), (5, 4, 8), (7, 3, 2)]:
        specs = [block_band_spec(r, world, h, b) for r in range(world)]
        rows = torch.cat([band_frame_rows(*sp, b) for sp in specs])
        assert sorted(rows.tolist()) == list(range(h)), (h, world, b)
        assert max(sp[1] for sp in specs) - min(sp[1] for sp in specs) <= b
    with pytest.raises(ValueError):
        block_band_spec(0, 2, 16, 3)


def test_split_band_spec_compositor():
    """The compositor split (bench.py --compositor): rank 0 renders no row, ranks 1..K-1 hold the
    (K-1)-way block-cyclic split; without it, block_band_spec."""
    from voxelraytracer_amd.tiles import band_frame_rows, block_band_spec, split_band_spec

    assert split_band_spec(2, 4, 1080, 16) == block_band_spec(2, 4, 1080, 16)
    for h, world, b in [(1080, 8, 16), (2160, 4, 16), (21, 3, 4), (18, 4, 1)]:
        specs = [split_band_spec(r, world, h, b, True) for r in range(world)]
        assert specs[0][1] == 0
        assert specs[1:] == [block_band_spec(r - 1, world - 1, h, b) for r in range(1, world)]
        rows = torch.cat([band_frame_rows(*sp, b) for sp in specs])
        assert sorted(rows.tolist()) == list(range(h)), (h, world, b)
    with pytest.raises(ValueError):
        split_band_spec(0, 2, 16, 4, True)


@pytest.mark.parametrize("world,lanes,row_block,mode", [(3, 2, 4, "f32"), (4, 1, 1, "f32"),
                                                        (3, 2, 2, "rgba8")])
def test_compositor_frames_match_single_process(built, world, lanes, row_block, mode):
    """Gathered frames with a compositor rank 0 (it renders nothing; ranks 1..K-1 split the frame,
    rank 0 assembles every frame): float frames, and the RGBA8 temporal sequence with dependent
    lanes (each renderer's history is its own band), equal the single-process frames bit for bit."""
    import oracle
    import voxelraytracer_amd as vrt

    n, w, h, frames, alpha = 16, 24, 18, 3, 0.5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, w, h, frames, q, mode, alpha,
                                              1, True, lanes, row_block, True)) for r in range(world)]
    for p in procs:
        p.start()
    got, _ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    vox = vrt.build_scene("glass_cube", n)
    cam = vrt.make_camera(w, h)
    hist = np.zeros((h, w, 4), np.uint8)
    assert len(got) == frames
    for t in range(frames):
        ref, _, _ = oracle.render(cam, vox, n, vrt.default_params(1, 2, time=float(t + 1),
                                                                  ray_noise=0.05))
        if mode == "rgba8":
            _, hist = oracle.temporal(ref, hist, alpha)
            assert np.array_equal(got[t], hist), t
        else:
            assert np.array_equal(got[t].view(np.uint32), ref.view(np.uint32)), t


@pytest.mark.parametrize("world,h,row_block,lanes", [(2, 16, 8, 2), (3, 21, 4, 2)])
def test_block_bands_without_per_frame_gather(built, world, h, row_block, lanes):
    """Block-cyclic bands kept on their ranks with frames in flight (bench.py's multi-GPU default:
    8-row blocks), incl. a ragged split (21 rows in blocks of 4 over 3 ranks: bands of 8, 8, 5
    rows): collect() assembles the single-process RGBA8 temporal sequence bit for bit."""
    import oracle
    import voxelraytracer_amd as vrt

    n, w, frames, alpha = 16, 20, 3, 0.5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, w, h, frames, q, "rgba8", alpha,
                                              1, False, lanes, row_block)) for r in range(world)]
    for p in procs:
        p.start()
    got, _ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    vox = vrt.build_scene("glass_cube", n)
    cam = vrt.make_camera(w, h)
    hist = np.zeros((h, w, 4), np.uint8)
    assert len(got) == frames
    for t in range(frames):
        rgba, _, _ = oracle.render(cam, vox, n, vrt.default_params(1, 2, time=float(t + 1),
                                                                   ray_noise=0.05))
        _, hist = oracle.temporal(rgba, hist, alpha)
        assert np.array_equal(got[t], hist), t
