"""Framebuffer tiling across the GPUs of one node, and frames in flight.

The per-pixel program has no halo and no inter-ray exchange, so a frame splits into row bands,
one per rank (one process per GPU). Bands are cyclic — rank r owns rows r, r+N, r+2N, ... — so
every rank gets the same mix of cheap sky rows and expensive geometry rows. With row_block = B
(ABI v11; bench.py's split frames use 16) rank r owns blocks r, r+N, ... of B adjacent rows instead,
so an 8x8 pixel wave covers 8 adjacent frame rows and its rays' walks stay as coherent as in the
whole frame (the slowest of 8 bands: C3 0.0150 -> 0.0139, C4 0.0274 -> 0.0237 ms per frame,
profiles/r03_s45, r03_s46); bands then differ by at most one block. Each rank renders its
band into HBM. The volume is replicated once per GPU (broadcast_volume). The only exchange is the
output: one gather of the bands to rank 0 per frame (gather=True, bench.py's default for N > 1:
SURVEY §8e's RCCL gather over xGMI; rank 0 re-interleaves the bands into the frame), or none — the
bands stay on their ranks (gather=False) and collect() gathers one frame when it is wanted.

Within a rank the band is rendered as P interleaved parts (global part q = s*N + r owns frame
rows q, q + N*P, ...), each on its own HIP stream, and — without the per-frame gather — L frames
may be in flight at once ("lanes"): frame k renders on lane k % L (P streams and an output buffer
of its own). A frame's last dispatch round leaves wave slots idle while its longest waves (the
exact-path and glass pixels, tens of microseconds) finish; the next frames' launches on the other
lanes fill them. At u_Alpha = 1 (the slider default, res/guis/header.xml:20) a frame does not read
its history (the RGB8 blend is the identity, tests/test_temporal_oracle.py), so consecutive frames
are independent (independent=True: no ordering between lanes at all). Otherwise part s of frame k
waits for part s of frame k-1 (its history rows) with one event. Measured on one MI355X
(scripts/diag/strong_pipe.py, profiles/r03_pipe/): C3's band at k = 8 GPUs takes 0.0416 ms per frame
with one lane of two parts and 0.0112 ms with four lanes of one part; the whole 1080p frame 0.0599 ms.

With one lane every part renders straight into its rows of the band buffer (a row-strided view;
the renderer's row pitch, ABI v4) and filters them in place against the same rows, which hold the
previous frame: no band buffers, no assembly copy. With several lanes a part reads its history
from the previous lane's buffer and writes its own.

With gather=True every frame's render, gather and (rank 0) assembly are enqueued on its lane's
stream, so frames in flight on the other lanes overlap the gather of this one, and a lane's band
buffer is rewritten only after the gather that read it (stream order; ABI v12). The exchange is
pluggable: GatherLib (the library's ncclGather on one RCCL communicator per lane + its assembly
kernel, bench.py's nccl runs: three C calls per frame, no cross-stream events) or GatherTorch
(torch.distributed.gather + index_copy_, synchronous per frame: the gloo tests). Bands are padded
to the largest band's rows so that every rank sends the same bytes. Bands are RGBA8 words when the
renderer runs the fused temporal filter + RGB8 store (main.cpp:363-393): 4 B per pixel on the wire.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def band_spec(rank: int, world: int, height: int):
    """(row0, rows, row_step) of rank's cyclic band; height must divide by world."""
    if height % world:
        raise ValueError(f"frame height {height} is not divisible by {world} ranks")
    return rank, height // world, world


def block_band_spec(rank: int, world: int, height: int, block: int):
    """(row0, rows, row_step) of rank's block-cyclic band (ABI v11's row_block form): blocks of
    `block` adjacent frame rows, rank r owns blocks r, r + world, ...; band row i is frame row
    row0 + (i // block) * row_step + i % block. The last block is short when height % block != 0,
    and bands differ by at most one block (no divisibility needed). block = 1 is band_spec's
    cyclic band. An 8x8 pixel wave of a block-8 band covers 8 adjacent frame rows, as in the whole
    frame, instead of 8 rows `world` apart (coherent walks: DESIGN.md §8)."""
    if block & (block - 1) or not 1 <= block <= 64:
        raise ValueError("block must be a power of two in [1, 64]")
    nb = -(-height // block)
    own = max(0, (nb - rank + world - 1) // world)
    rows = own * block
    if own and (nb - 1) % world == rank:
        rows -= nb * block - height
    return rank * block, rows, world * block


def split_band_spec(rank: int, world: int, height: int, block: int, compositor: bool = False):
    """(row0, rows, row_step) of rank's band of the frame split. compositor=False: block_band_spec
    over all `world` ranks. compositor=True (world >= 3): rank 0 renders no rows — it receives and
    assembles every frame — and ranks 1..world-1 split the frame block-cyclically among themselves
    (rank r renders renderer r - 1's band of a (world - 1)-way split): with every frame gathered,
    rank 0's exchange share (packing, the collective, the assembly of the whole frame) is worth
    about one 8-way C3 band's render."""
    if not compositor:
        return block_band_spec(rank, world, height, block)
    if world < 3:
        raise ValueError("a compositor rank needs at least two renderers")
    if rank == 0:
        return 0, 0, (world - 1) * block
    return block_band_spec(rank - 1, world - 1, height, block)


def band_frame_rows(row0: int, rows: int, row_step: int, block: int = 1) -> torch.Tensor:
    """Frame row of every band row of a (block-)cyclic band, as an int64 index tensor."""
    i = torch.arange(rows, dtype=torch.int64)
    return row0 + (i // block) * row_step + i % block


def part_spec(rank: int, world: int, part: int, parts: int, height: int):
    """(row0, rows, row_step) of part `part` of rank's band: global part q = part*world + rank
    owns frame rows q, q + world*parts, ...; height must divide by world*parts."""
    total = world * parts
    if height % total:
        raise ValueError(f"frame height {height} is not divisible by {world} ranks x {parts} parts")
    return part * world + rank, height // total, total


def assemble_cyclic(bands: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bands[world, rows, W, C] (rank-major) -> frame[rows*world, W, C] with frame row i*world+r
    = bands[r, i]."""
    world, rows, w, c = bands.shape
    if out is None:
        out = torch.empty((rows * world, w, c), dtype=bands.dtype, device=bands.device)
    out.view(rows, world, w, c).copy_(bands.permute(1, 0, 2, 3))
    return out


def assemble_parts(gathered: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """gathered[world, parts, rows, W, C] -> frame[rows*parts*world, W, C] with frame row
    j*(world*parts) + part*world + rank = gathered[rank, part, j]."""
    world, parts, rows, w, c = gathered.shape
    if out is None:
        out = torch.empty((rows * parts * world, w, c), dtype=gathered.dtype,
                          device=gathered.device)
    out.view(rows, parts, world, w, c).copy_(gathered.permute(2, 1, 0, 3, 4))
    return out


def row_pitch(t: torch.Tensor) -> int:
    """Pixels from one row to the next of a [rows, W, C] band tensor that render_band receives
    (it may be a row-strided view into the frame): the renderer's `pitch` argument."""
    if t.dim() != 3 or t.stride(2) != 1 or t.stride(1) != t.shape[2]:
        raise ValueError("band tensors are [rows, W, C] with contiguous pixels")
    return t.stride(0) // t.stride(1)


def broadcast_volume(vox: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    """Replicate the N^3 volume (uint8 tensor on this rank's device) from `src` to every rank."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(vox, src, group=group)
    return vox


class GatherTorch:
    """Per-frame exchange through torch.distributed: dist.gather of every rank's padded band to rank
    0, then rank 0's re-interleave (index_copy_ into the frame). Synchronous per frame (a gloo
    gather of CUDA tensors blocks the host; with nccl, work.wait() orders the lane stream after the
    collective): no collective is left outstanding across frames. The exchange of the gloo tests
    (two ranks sharing one GPU, where RCCL cannot run) and of CPU tiling."""

    def __init__(self, group=None):
        self.group = group

    def run(self, tiler, slot: int) -> None:
        band = tiler.bufs[slot]
        glist = list(tiler.gathered[slot].unbind(0)) if tiler.rank == 0 else None
        dist.gather(band, glist, dst=0, group=self.group)
        if tiler.rank == 0:
            g = tiler.gathered[slot]
            tiler.frames[slot].index_copy_(0, tiler.asm_index, g.view(-1, *g.shape[2:]))


class GatherLib:
    """Per-frame exchange through the C-ABI (ABI v12): ncclGather of the padded band to rank 0 on
    one RCCL communicator per lane (vrt_gather_band_async) and, on rank 0, the assembly kernel
    (vrt_assemble_blocks_async) — both enqueued on the lane's stream right after its render, so
    that the next frames on the other lanes overlap them and no event crosses streams. RGBA8 bands
    cross xGMI in the RGB8 wire format (wire="rgb8", the default for them: the A byte is always
    255, so 3 of 4 bytes; vrt_pack_rgb8_async before the gather, the assembly unpacks): rank 0's
    ingress bounds the gather. The communicators are joined (vrt_comm_join) with ids rank 0
    creates and `share_ids` distributes (bench.py: a broadcast over the job's process group)."""

    def __init__(self, renderer, lanes: int, world: int, rank: int, share_ids, wire: str = "rgb8"):
        import voxelraytracer_amd as vrt

        ids = [vrt.comm_unique_id() for _ in range(lanes)] if rank == 0 else None
        ids = share_ids(ids, lanes)
        renderer.comm_join(ids, world, rank)
        self.ren, self.lanes, self.wire, self.args = renderer, lanes, wire, None
        # timing (bench.py, after its timed region): None, or a list collecting per exchanged frame
        # the events (start, after the pack + ncclGather, after rank 0's assembly) on its lane stream
        self.timing = None

    def _setup(self, tiler) -> None:
        self.rgb8 = (self.wire == "rgb8" and tiler.dtype == torch.uint8 and tiler.channels == 4
                     and tiler.width % 4 == 0)
        self.words = tiler.width * tiler.channels * tiler.dtype.itemsize // 4
        self.packed = self.gpacked = None
        dev = tiler.bufs[0].device
        if self.rgb8:   # per frame slot: the packed band, and (rank 0) the gathered packed bands
            px = tiler.rmax * tiler.width
            self.packed = [torch.empty(px * 3, dtype=torch.uint8, device=dev) for _ in range(tiler.slots)]
            if tiler.rank == 0:
                self.gpacked = [torch.empty(tiler.world * px * 3, dtype=torch.uint8, device=dev)
                                for _ in range(tiler.slots)]
        self.tstreams = [tiler.part_streams[g // tiler.batch][0] for g in range(tiler.slots)]
        self.args = []
        for g in range(tiler.slots):   # (band, pixels, packed, gathered, frame, stream, communicator)
            self.args.append((tiler.bufs[g].data_ptr(), tiler.bufs[g].numel() // tiler.channels,
                              self.packed[g].data_ptr() if self.rgb8 else 0,
                              (self.gpacked[g] if self.rgb8 else tiler.gathered[g]).data_ptr()
                              if tiler.rank == 0 else 0,
                              tiler.frames[g].data_ptr() if tiler.rank == 0 else 0,
                              tiler.part_streams[g // tiler.batch][0].cuda_stream,
                              (g // tiler.batch) % self.lanes))

    def bytes_per_rank(self, tiler) -> int:
        """Bytes every rank sends per frame."""
        if self.args is None:
            self._setup(tiler)
        px = tiler.rmax * tiler.width
        return px * 3 if self.rgb8 else px * tiler.channels * tiler.dtype.itemsize

    def run(self, tiler, slot: int) -> None:
        if self.args is None:
            self._setup(tiler)
        band, px, packed, gath, frame, st, comm = self.args[slot]
        evs = None
        if self.timing is not None:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            evs[0].record(self.tstreams[slot])   # completes when the frame's render has
        # a compositor rank 0 renders no rows: its chunk of the gather is not packed and not
        # assembled (the bands of ranks 1.. start one padded band into the gathered buffer)
        nb = tiler.world - 1 if tiler.compositor else tiler.world
        if self.rgb8:
            if not (tiler.compositor and tiler.rank == 0):
                self.ren.pack_rgb8_async(band, px, packed, st)
            self.ren.gather_band_async(comm, packed, px * 3, gath, st)
            if evs:
                evs[1].record(self.tstreams[slot])
            if tiler.rank == 0:
                g0 = gath + (px * 3 if tiler.compositor else 0)
                self.ren.assemble_blocks_rgb8_async(g0, nb, tiler.rmax, tiler.width, tiler.height,
                                                    tiler.row_block, frame, tiler.width, st)
        else:
            bb = px * tiler.channels * tiler.dtype.itemsize
            self.ren.gather_band_async(comm, band, bb, gath, st)
            if evs:
                evs[1].record(self.tstreams[slot])
            if tiler.rank == 0:
                self.ren.assemble_blocks_async(gath + (bb if tiler.compositor else 0), nb, tiler.rmax,
                                               self.words, tiler.height, tiler.row_block, frame, self.words, st)
        if evs:
            evs[2].record(self.tstreams[slot])
            self.timing.append(evs)


class GatherRehearsal(GatherLib):
    """Rank 0's local share of the per-frame exchange, for a one-GPU rehearsal of rank 0 of a
    K-way split (bench.py --rehearse-gather): every frame's own band is packed to the RGB8 wire
    format and the K gathered bands are assembled into the frame (vrt_assemble_blocks_rgb8_async)
    on the frame's lane stream, exactly as GatherLib does after its ncclGather; the collective
    itself (the other ranks' bands arriving over xGMI) is not rehearsed, so the gathered buffer
    holds whatever it held. What it times: the packing and assembly work rank 0 adds to its own
    rendering."""

    def __init__(self, renderer, lanes: int):
        self.ren, self.lanes, self.wire, self.args = renderer, lanes, "rgb8", None
        self.timing = None

    def run(self, tiler, slot: int) -> None:
        if self.args is None:
            self._setup(tiler)
        band, px, packed, gath, frame, st, _ = self.args[slot]
        if not self.rgb8:
            raise ValueError("the gather rehearsal is for RGBA8 bands (RGB8 wire)")
        nb = tiler.world - 1 if tiler.compositor else tiler.world
        if not tiler.compositor:
            self.ren.pack_rgb8_async(band, px, packed, st)
        self.ren.assemble_blocks_rgb8_async(gath + (px * 3 if tiler.compositor else 0), nb, tiler.rmax,
                                            tiler.width, tiler.height, tiler.row_block, frame, tiler.width, st)


class FrameTiler:
    """Renders a sequence of frames across `world` ranks, `parts` streams per lane, `lanes`
    frames in flight per rank.

    render_band(row0, rows, row_step, out, prev) must enqueue the render of one part into `out`
    ([rows, W, channels] of `dtype` on `device`; a row-strided view, see row_pitch) on the CURRENT
    stream (the HIP kernel through the C-ABI, or the oracle in CPU tests); `prev` holds that
    part's rows of the previous frame (the temporal history; zeros before the first frame; with
    one lane it is `out` itself: each pixel is read before it is written). Block-cyclic bands
    (row_block > 1, and every gathered band) receive row_block= as well.
    frame() enqueues the next frame. With gather=False (or one rank) it returns this rank's band
    of it ([rows, W, C], the whole frame with one rank); collect() (after finish()) assembles the
    last frame on rank 0 with one gather. With several ranks and gather=True every frame is
    gathered to rank 0 and re-interleaved there by `exchange` (GatherTorch by default; GatherLib
    for the library's RCCL path), in the frame's lane stream: frame() returns the new frame on
    rank 0 (complete once that stream is synchronised) and None elsewhere. A returned band or
    frame stays valid until `lanes` more frames are enqueued. finish() makes the current stream
    wait for every frame enqueued so far and returns the last frame (rank 0 with gather) or band.
    compositor=True (gathered block-cyclic bands, world >= 3): rank 0 renders no band — every
    frame is split over ranks 1..world-1 (split_band_spec) and rank 0 only receives and assembles.
    independent=True declares that render_band does not read `prev` (u_Alpha = 1): frames on
    different lanes are then not ordered at all.
    launch (optional, CUDA): the lean form of render_band, launch(row0, rows, row_step,
    out_ptr, prev_ptr, pitch, stream_handle) with device pointers, the row pitch in pixels and the
    part's HIP stream; frames whose lanes need no event ordering (one lane, or independent) then
    enqueue from precomputed arguments with no torch stream switches or tensor views (~4 us per
    launch on the host instead of ~20: a band of a k-GPU split at k = 8 renders in ~11 us).
    batch > 1 (independent frames, one part, launch_batch given): `batch` consecutive frames of a
    lane are rendered by ONE launch, launch_batch(row0, rows, row_step, out_ptrs, pitch, stream)
    (vrt_render_temporal_batch_async), enqueued when the batch's last frame is requested (finish()
    enqueues a partial batch); each frame has its own buffer (slot), exchanged after the launch. A
    lane then holds `batch` frames in flight.
    """

    def __init__(self, width: int, height: int, render_band: Callable, device, group=None,
                 channels: int = 4, dtype=torch.float32, parts: int = 1, gather: bool = True,
                 lanes: int = 1, independent: bool = False, launch: Optional[Callable] = None,
                 world: Optional[int] = None, rank: Optional[int] = None, row_block: int = 1,
                 exchange=None, batch: int = 1, launch_batch: Optional[Callable] = None,
                 compositor: bool = False):
        # world / rank: override the process group's (one process rehearsing rank `rank` of a
        # `world`-way split on one GPU; no exchange may then be requested)
        self.world = world or (dist.get_world_size(group) if dist.is_initialized() else 1)
        self.rank = rank if rank is not None else (dist.get_rank(group) if dist.is_initialized() else 0)
        if world is not None and gather and not (isinstance(exchange, GatherRehearsal) and rank == 0):
            raise ValueError("a rehearsed split keeps its band (gather=False), except rank 0 with "
                             "GatherRehearsal (its local share of the exchange)")
        if lanes < 1:
            raise ValueError("lanes >= 1")
        if batch < 1 or (batch > 1 and (not independent or parts != 1 or launch_batch is None)):
            raise ValueError("frame batches need independent frames, one part and launch_batch")
        self.batch = batch
        self.slots = lanes * batch   # frame buffers: slot = lane * batch + frame of the batch
        self.pending = 0             # frames of the current batch requested but not yet launched
        self.group = group
        self.width, self.height, self.parts = width, height, parts
        self.row_block = row_block
        self.gather = gather and self.world > 1
        # split_band_spec's compositor split: rank 0 renders nothing and assembles the frames
        self.compositor = compositor
        if compositor and not (row_block > 1 or self.gather):
            raise ValueError("the compositor split is a block-cyclic split")
        if row_block > 1 or self.gather:
            # block-cyclic band (row_block 1: cyclic rows), one part per lane; bands may be unequal
            if parts != 1:
                raise ValueError("block-cyclic and gathered bands are one part per lane (parts=1)")
            self.row0, self.rows, self.step = split_band_spec(self.rank, self.world, height, row_block,
                                                              compositor)
            self.specs = [(self.row0, self.rows, self.step)]
        else:
            self.row0, self.rows, self.step = band_spec(self.rank, self.world, height)
            self.specs = [part_spec(self.rank, self.world, s, parts, height) for s in range(parts)]
        # render_band / launch receive row_block= for block-cyclic (and gathered) bands
        self.block_kw = {"row_block": row_block} if (row_block > 1 or self.gather) else {}
        self.rows_p = self.specs[0][1]
        self.render_band = render_band
        self.cuda = torch.device(device).type == "cuda"
        self.lanes, self.independent = lanes, independent
        self.channels, self.dtype = channels, dtype
        self.exchange = None
        self.exchange_on = True   # bench.py's render-only pass switches the per-frame gather off
        # per lane: exchanges enqueued and the sum of their frame indices. A lane's collective runs
        # on that lane's own communicator in enqueue order, so every rank must enqueue the same
        # frames on every lane: exchange_log() is compared across ranks (bench.py)
        self.xlog = [[0, 0] for _ in range(lanes)]
        self.launch_batch = launch_batch
        self.latest = None
        if self.gather:
            # every rank's band padded to the largest band's rows: equal gather sizes
            specs = [split_band_spec(r, self.world, height, row_block, compositor) for r in range(self.world)]
            self.rmax = max(sp[1] for sp in specs)
            self.bufs = [torch.zeros((self.rmax, width, channels), dtype=dtype, device=device)
                         for _ in range(self.slots)]
            self.gathered = self.frames = None
            if self.rank == 0:
                self.gathered = [torch.empty((self.world, self.rmax, width, channels), dtype=dtype,
                                             device=device) for _ in range(self.slots)]
                # frame row of every gathered row; padding rows land in a scratch row `height`
                idx = torch.full((self.world, self.rmax), height, dtype=torch.int64)
                for r, (r0, rows, step) in enumerate(specs):
                    idx[r, :rows] = band_frame_rows(r0, rows, step, row_block)
                self.asm_index = idx.reshape(-1).to(device)
                self.frames = [torch.zeros((height + 1, width, channels), dtype=dtype, device=device)
                               for _ in range(self.slots)]
            self.exchange = exchange or GatherTorch(group)
        else:
            # this rank's band per lane; part s renders band rows s, s + parts, ... in place
            self.bufs = [torch.zeros((self.rows, width, channels), dtype=dtype, device=device)
                         for _ in range(self.slots)]
        self.part_streams = ([[torch.cuda.Stream(device=device) for _ in range(parts)]
                              for _ in range(lanes)]
                             if self.cuda and (parts > 1 or lanes > 1 or self.gather or batch > 1) else None)
        self.part_done = [[None] * parts for _ in range(lanes)]   # dependent lanes: frame events
        self.fresh = True   # the streams must first wait for the current stream's work
        self.plan = None   # lean launches: per lane, per part (row0, rows, step, out, prev, pitch, stream)
        if batch > 1:
            if self.part_streams is None:
                raise ValueError("frame batches need CUDA streams")
            row0, rows, step = self.specs[0]
            self.plan = []   # per lane: (row0, rows, step, out pointers of its slots, pitch, stream)
            for g in range(lanes):
                outs = [self.part_rows(self.bufs[g * batch + j], 0) for j in range(batch)]
                self.plan.append((row0, rows, step, [o.data_ptr() for o in outs], row_pitch(outs[0]),
                                  self.part_streams[g][0].cuda_stream))
        elif launch is not None and self.part_streams is not None and (lanes == 1 or independent):
            self.launch = launch
            self.plan = []
            for g in range(lanes):
                out_b, prev_b = self.bufs[g], self.bufs[(g - 1) % lanes]
                row = []
                for q, (row0, rows, step) in enumerate(self.specs):
                    o, pv = self.part_rows(out_b, q), self.part_rows(prev_b, q)
                    row.append((row0, rows, step, o.data_ptr(), pv.data_ptr(), row_pitch(o),
                                self.part_streams[g][q].cuda_stream))
                self.plan.append(row)
        self.k = 0

    # ---- helpers ---------------------------------------------------------------------------
    def part_rows(self, buf: torch.Tensor, s: int) -> torch.Tensor:
        """Part s's rows of a band buffer (band rows s, s + parts, ...; a gathered band's padding
        rows excluded)."""
        if self.gather:
            return buf[:self.rows]
        return buf.view(self.rows_p, self.parts, self.width, -1)[:, s]

    def slot_of(self, k: int) -> int:
        """The buffer slot of frame k (its lane's batch position)."""
        return ((k // self.batch) % self.lanes) * self.batch + k % self.batch

    def last(self) -> torch.Tensor:
        """This rank's band buffer of the last frame enqueued (its band rows)."""
        b = self.bufs[self.slot_of(self.k - 1)]
        return b[:self.rows] if self.gather else b

    def next_stream(self):
        """The HIP stream the next frame's (first) launch is enqueued on (CUDA), or None."""
        if self.part_streams is None:
            return torch.cuda.current_stream() if self.cuda else None
        return self.part_streams[(self.k // self.batch) % self.lanes][0]

    def _render_parts(self, lane: int, band: torch.Tensor, prev: torch.Tensor):
        """Enqueue every part of the next frame on `lane` (and its exchange). Returns the parts'
        completion events (CUDA streams, dependent lanes)."""
        if self.part_streams is None:
            for s, (row0, rows, step) in enumerate(self.specs):
                if rows:
                    self.render_band(row0, rows, step, self.part_rows(band, s), self.part_rows(prev, s),
                                     **self.block_kw)
            if self.gather and self.exchange_on:
                self._log_exchange(lane)
                self.exchange.run(self, lane)
            return None
        cur = torch.cuda.current_stream()
        if self.fresh:
            for ln in self.part_streams:
                for st in ln:
                    st.wait_stream(cur)
            self.fresh = False
        dep = self.lanes > 1 and not self.independent
        prev_lane = (lane - 1) % self.lanes
        events = []
        for s, (row0, rows, step) in enumerate(self.specs):
            st = self.part_streams[lane][s]
            with torch.cuda.stream(st):
                if dep and self.part_done[prev_lane][s] is not None:
                    st.wait_event(self.part_done[prev_lane][s])   # the history rows of part s
                if rows:
                    self.render_band(row0, rows, step, self.part_rows(band, s), self.part_rows(prev, s),
                                     **self.block_kw)
                if self.gather and self.exchange_on:
                    if s == 0:
                        self._log_exchange(lane)
                    self.exchange.run(self, lane)
                ev = st.record_event() if dep else None
                self.part_done[lane][s] = ev
                events.append(ev)
        return events

    def _log_exchange(self, lane: int, k: Optional[int] = None) -> None:
        self.xlog[lane][0] += 1
        self.xlog[lane][1] += self.k - 1 if k is None else k   # the index of the frame being enqueued

    def _flush_batch(self) -> None:
        """Launch the pending frames of the current batch (one launch) and their exchanges."""
        n = self.pending
        if n == 0:
            return
        self.pending = 0
        k0 = self.k - n
        lane = (k0 // self.batch) % self.lanes
        if self.fresh:
            cur = torch.cuda.current_stream()
            for ln in self.part_streams:
                for st in ln:
                    st.wait_stream(cur)
            self.fresh = False
        row0, rows, step, outs, pitch, stream = self.plan[lane]
        if rows:   # a compositor rank 0 renders nothing
            self.launch_batch(row0, rows, step, outs[:n], pitch, stream, **self.block_kw)
        if self.gather and self.exchange_on:
            for j in range(n):
                self._log_exchange(lane, k0 + j)
                slot = lane * self.batch + j
                if isinstance(self.exchange, GatherLib):
                    self.exchange.run(self, slot)
                else:
                    with torch.cuda.stream(self.part_streams[lane][0]):
                        self.exchange.run(self, slot)

    def exchange_log(self):
        """Per lane [exchanges enqueued, sum of their frame indices] (a flat list of 2 x lanes ints):
        equal on every rank iff every rank enqueued the same frames' gathers on every lane."""
        return [v for row in self.xlog for v in row]

    # ---- pipeline --------------------------------------------------------------------------
    def frame(self) -> Optional[torch.Tensor]:
        if self.batch > 1:   # frame batches: one launch per `batch` frames of a lane
            slot = self.slot_of(self.k)
            self.k += 1
            self.pending += 1
            if self.pending == self.batch:
                self._flush_batch()
            if not self.gather:
                return self.bufs[slot]
            self.latest = self.frames[slot][:self.height] if self.rank == 0 else None
            return self.latest
        lane = self.k % self.lanes
        self.k += 1
        if self.plan is not None:   # lean launches from precomputed arguments
            if self.fresh:
                cur = torch.cuda.current_stream()
                for ln in self.part_streams:
                    for st in ln:
                        st.wait_stream(cur)
                self.fresh = False
            for args in self.plan[lane]:
                if args[1]:
                    self.launch(*args, **self.block_kw)
            if self.gather and self.exchange_on:
                self._log_exchange(lane)
                if isinstance(self.exchange, GatherLib):
                    self.exchange.run(self, lane)
                else:
                    with torch.cuda.stream(self.part_streams[lane][0]):
                        self.exchange.run(self, lane)
        else:
            self._render_parts(lane, self.bufs[lane], self.bufs[(self.k - 2) % self.lanes])
        if not self.gather:
            return self.bufs[lane]
        self.latest = self.frames[lane][:self.height] if self.rank == 0 else None
        return self.latest

    def collect(self) -> Optional[torch.Tensor]:
        """After finish(): one gather of every rank's band of the last frame to rank 0 through the
        process group, re-interleaved into the whole frame (returned on rank 0, None elsewhere);
        e.g. to display the last frame of bands kept on their ranks, or to check a gathered frame
        against an independent assembly. Synchronous."""
        band = self.last().contiguous()
        if self.world == 1:
            return band
        if self.row_block == 1 and not self.gather:   # equal cyclic bands (band_spec)
            glist = ([torch.empty_like(band) for _ in range(self.world)] if self.rank == 0 else None)
            dist.gather(band, glist, dst=0, group=self.group)
            return assemble_cyclic(torch.stack(glist)) if self.rank == 0 else None
        # block-cyclic bands may differ by one block: gather them padded to the largest
        specs = [split_band_spec(r, self.world, self.height, self.row_block, self.compositor)
                 for r in range(self.world)]
        rmax = max(sp[1] for sp in specs)
        pad = band.new_zeros((rmax,) + tuple(band.shape[1:]))
        pad[:band.shape[0]] = band
        glist = ([torch.empty_like(pad) for _ in range(self.world)] if self.rank == 0 else None)
        dist.gather(pad, glist, dst=0, group=self.group)
        if self.rank != 0:
            return None
        out = band.new_empty((self.height,) + tuple(band.shape[1:]))
        for r, (row0, rows, step) in enumerate(specs):
            out[band_frame_rows(row0, rows, step, self.row_block).to(out.device)] = glist[r][:rows]
        return out

    def mark_idle(self) -> None:
        """Declare the device idle (the caller has just synchronised it): the next frame's streams
        need not wait for the current stream's work, so they start without cross-queue waits."""
        self.fresh = False

    def lane_streams(self):
        """The HIP streams the frames are enqueued on (empty without part streams)."""
        return [st for ln in (self.part_streams or ()) for st in ln]

    def flush(self) -> None:
        """Enqueue the frames of a partial batch now (frame batches; no-op otherwise): e.g. before
        recording an event after the last frame of a timed region."""
        if self.batch > 1:
            self._flush_batch()

    def finish(self) -> Optional[torch.Tensor]:
        if self.batch > 1:
            self._flush_batch()   # a partial batch
        if self.cuda:
            cur = torch.cuda.current_stream()
            for ln in self.part_streams or ():
                for st in ln:
                    cur.wait_stream(st)
        self.fresh = True
        if self.gather:
            return self.latest
        return self.last()
