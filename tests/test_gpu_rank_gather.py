"""The library's one-process-per-GPU exchange (ABI v12) on the one-GPU box: RCCL communicators
joined from unique ids (vrt_comm_unique_id / vrt_comm_join, a one-rank job here), ncclGather of a
band through vrt_gather_band_async, and the assembly kernel (vrt_assemble_blocks_async) that
re-interleaves k gathered block-cyclic bands into the frame — checked byte for byte against the
band placement of tiles.band_frame_rows. Also tiles.GatherLib, the exchange bench.py's nccl runs
use, through a one-rank job. Between distinct GPUs the gather runs only in the driver's runs."""
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def reference_frame(bands: torch.Tensor, k: int, height: int, block: int) -> torch.Tensor:
    from voxelraytracer_amd.tiles import band_frame_rows, block_band_spec

    frame = torch.zeros((height,) + tuple(bands.shape[2:]), dtype=bands.dtype)
    for j in range(k):
        row0, rows, step = block_band_spec(j, k, height, block)
        frame[band_frame_rows(row0, rows, step, block)] = bands[j, :rows].cpu()
    return frame


@pytest.mark.parametrize("k,width,height,block", [(3, 40, 53, 16), (8, 1920, 1080, 16), (8, 3840, 2160, 16),
                                                  (2, 37, 9, 1), (5, 64, 100, 4)])
def test_assemble_blocks_matches_band_placement(built, k, width, height, block):
    import voxelraytracer_amd as vrt

    plan, cap = vrt.block_band_plan(height, k, block)
    g = torch.Generator().manual_seed(k * 1000 + width)
    bands = torch.randint(0, 256, (k, cap, width, 4), dtype=torch.uint8, generator=g).cuda()
    frame = torch.full((height, width, 4), 7, dtype=torch.uint8, device="cuda")
    with vrt.Renderer(0) as ren:
        st = torch.cuda.current_stream().cuda_stream
        ren.assemble_blocks_async(bands.data_ptr(), k, cap, width, height, block, frame.data_ptr(), width, st)
        torch.cuda.synchronize()
        with pytest.raises(vrt.VrtError):   # a band slice too small for the largest band
            ren.assemble_blocks_async(bands.data_ptr(), k, cap - 1, width, height, block, frame.data_ptr(),
                                      width, st)
    assert torch.equal(frame.cpu(), reference_frame(bands, k, height, block))


@pytest.mark.parametrize("k,width,height,block", [(3, 40, 53, 16), (8, 3840, 2160, 16), (2, 36, 9, 1)])
def test_rgb8_wire_assembly_matches_rgba8(built, k, width, height, block):
    """RGB8 wire format: pack each band (vrt_pack_rgb8_async), assemble from the packed bands
    (vrt_assemble_blocks_rgb8_async): the frame equals the RGBA8 assembly of the same bands."""
    import voxelraytracer_amd as vrt

    plan, cap = vrt.block_band_plan(height, k, block)
    g = torch.Generator().manual_seed(7 * k + width)
    bands = torch.randint(0, 256, (k, cap, width, 4), dtype=torch.uint8, generator=g)
    bands[..., 3] = 255   # pack_rgb8's A byte
    bands = bands.cuda()
    packed = torch.zeros(k * cap * width * 3, dtype=torch.uint8, device="cuda")
    frame = torch.zeros((height, width, 4), dtype=torch.uint8, device="cuda")
    with vrt.Renderer(0) as ren:
        st = torch.cuda.current_stream().cuda_stream
        for j in range(k):
            ren.pack_rgb8_async(bands[j].data_ptr(), cap * width, packed[j * cap * width * 3:].data_ptr(), st)
        ren.assemble_blocks_rgb8_async(packed.data_ptr(), k, cap, width, height, block, frame.data_ptr(), width, st)
        torch.cuda.synchronize()
    assert torch.equal(packed.view(k, cap, width, 3).cpu(), bands[..., :3].cpu())
    assert torch.equal(frame.cpu(), reference_frame(bands, k, height, block))


@pytest.mark.parametrize("wire,batch", [("rgb8", 1), ("rgba8", 1), ("rgb8", 3)])
def test_rank_comm_gather_one_rank(built, wire, batch):
    """GatherLib per frame slot (frame batches: `batch` slots per lane, each gathered on its lane's
    communicator and stream)."""
    import voxelraytracer_amd as vrt
    from voxelraytracer_amd.tiles import GatherLib

    w, h, block, lanes = 96, 40, 16, 2
    slots = lanes * batch
    with vrt.Renderer(0) as ren:
        ex = GatherLib(ren, lanes, 1, 0, lambda ids, n: ids, wire=wire)   # one rank: the ids stay here
        st = [torch.cuda.Stream() for _ in range(lanes)]
        bufs = [torch.randint(0, 256, (h, w, 4), dtype=torch.uint8, device="cuda") for _ in range(slots)]
        for b in bufs:
            b[..., 3] = 255   # rendered RGBA8 words: A = 255
        tiler = types.SimpleNamespace(
            width=w, height=h, channels=4, dtype=torch.uint8, world=1, rank=0, rmax=h, row_block=block,
            lanes=lanes, slots=slots, batch=batch, bufs=bufs, part_streams=[[s] for s in st], compositor=False,
            gathered=[torch.zeros((1, h, w, 4), dtype=torch.uint8, device="cuda") for _ in range(slots)],
            frames=[torch.zeros((h + 1, w, 4), dtype=torch.uint8, device="cuda") for _ in range(slots)])
        for slot in range(slots):
            ex.run(tiler, slot)
        torch.cuda.synchronize()
        assert ex.rgb8 == (wire == "rgb8")
        assert [a[-1] for a in ex.args] == [(g // batch) % lanes for g in range(slots)]   # lane communicators
        for slot in range(slots):
            if not ex.rgb8:
                assert torch.equal(tiler.gathered[slot][0], bufs[slot])  # ncclGather of one rank
            assert torch.equal(tiler.frames[slot][:h], bufs[slot])       # assembly of one band
        with pytest.raises(vrt.VrtError):
            ren.gather_band_async(lanes, bufs[0].data_ptr(), bufs[0].numel(), 0, 0)  # no such comm
        with pytest.raises(vrt.VrtError):   # joined once per context
            ren.comm_join([vrt.comm_unique_id()], 1, 0)


def test_compositor_assembly_skips_rank0_chunk(built):
    """A compositor rank 0 (tiles.split_band_spec): the gathered buffer's chunk 0 is rank 0's
    unused send; the frame is assembled from chunks 1..K-1 as a (K-1)-way block-cyclic split
    (GatherRehearsal runs GatherLib's assembly without the collective)."""
    import voxelraytracer_amd as vrt
    from voxelraytracer_amd.tiles import GatherRehearsal

    k, w, h, block = 4, 96, 70, 16
    plan, cap = vrt.block_band_plan(h, k - 1, block)
    g = torch.Generator().manual_seed(11)
    bands = torch.randint(0, 256, (k - 1, cap, w, 4), dtype=torch.uint8, generator=g)
    bands[..., 3] = 255
    gpacked = torch.cat([torch.full((1, cap, w, 3), 9, dtype=torch.uint8), bands[..., :3]]).reshape(-1).cuda()
    with vrt.Renderer(0) as ren:
        ex = GatherRehearsal(ren, 1)
        st = torch.cuda.Stream()
        tiler = types.SimpleNamespace(
            width=w, height=h, channels=4, dtype=torch.uint8, world=k, rank=0, rmax=cap, row_block=block,
            lanes=1, slots=1, batch=1, compositor=True, part_streams=[[st]],
            bufs=[torch.zeros((cap, w, 4), dtype=torch.uint8, device="cuda")],
            gathered=[None], frames=[torch.zeros((h + 1, w, 4), dtype=torch.uint8, device="cuda")])
        ex._setup(tiler)
        ex.gpacked[0].copy_(gpacked)
        ex.run(tiler, 0)
        torch.cuda.synchronize()
    assert torch.equal(tiler.frames[0][:h].cpu(), reference_frame(bands, k - 1, h, block))
