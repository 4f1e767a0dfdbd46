"""Framebuffer tiling across the GPUs of one node, and frames in flight.

The per-pixel program has no halo and no inter-ray exchange, so a frame splits into row bands,
one per rank (one process per GPU). Bands are cyclic — rank r owns rows r, r+N, r+2N, ... — so
every rank gets the same mix of cheap sky rows and expensive geometry rows. With row_block = B
(ABI v11; bench.py's split frames use 16) rank r owns blocks r, r+N, ... of B adjacent rows instead,
so an 8x8 pixel wave covers 8 adjacent frame rows and its rays' walks stay as coherent as in the
whole frame (the slowest of 8 bands: C3 0.0150 -> 0.0139, C4 0.0274 -> 0.0237 ms per frame,
profiles/r03_s45, r03_s46); bands then differ by at most one block. Each rank renders its
band into HBM. The volume is replicated once per GPU (broadcast_volume). The only exchange is the
output: either one gather of the bands to rank 0 per frame (gather=True: RCCL over xGMI with the
"nccl" backend, gloo on CPU for tests; rank 0 re-interleaves), or none — the bands stay on their
ranks (gather=False, bench.py's default for N > 1) and collect() gathers one frame when the whole
frame is wanted (SURVEY §8e's gather is output delivery, not part of the per-pixel path).

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

gather=True double-buffers the band so that the gather of frame k overlaps the render of frame
k+1 (one lane only). Bands are RGBA8 words when the renderer runs the fused temporal filter + RGB8
store (the reference's stored frame format, main.cpp:363-393): 4 B per pixel on the wire.
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


class FrameTiler:
    """Renders a sequence of frames across `world` ranks, `parts` streams per lane, `lanes`
    frames in flight per rank.

    render_band(row0, rows, row_step, out, prev) must enqueue the render of one part into `out`
    ([rows, W, channels] of `dtype` on `device`; a row-strided view, see row_pitch) on the CURRENT
    stream (the HIP kernel through the C-ABI, or the oracle in CPU tests); `prev` holds that
    part's rows of the previous frame (the temporal history; zeros before the first frame; with
    one lane it is `out` itself: each pixel is read before it is written).
    frame() enqueues the next frame; with gather=False (or one rank) it returns this rank's band
    of it ([rows, W, C], the whole frame with one rank); with several ranks and gather=True the
    gather is issued asynchronously and rank 0 returns the PREVIOUS frame, assembled on
    `self.assembly_stream` (None on the first call and on other ranks). finish() makes the current
    stream wait for every frame enqueued so far and returns the last frame (band) on rank 0 (the
    last band elsewhere with gather=False); collect() (gather=False) assembles the last frame on
    rank 0 with one gather. A returned band stays valid until `lanes` more frames are enqueued;
    synchronise the device before reading it. independent=True declares that render_band does
    not read `prev` (u_Alpha = 1): frames on different lanes are then not ordered at all.
    launch (optional, CUDA): the lean form of render_band, launch(row0, rows, row_step,
    out_ptr, prev_ptr, pitch, stream_handle) with device pointers, the row pitch in pixels and the
    part's HIP stream; frames whose lanes need no event ordering (one lane, or independent) then
    enqueue from precomputed arguments with no torch stream switches or tensor views (~4 us per
    launch on the host instead of ~20: a band of a k-GPU split at k = 8 renders in ~11 us).
    """

    def __init__(self, width: int, height: int, render_band: Callable, device, group=None,
                 channels: int = 4, dtype=torch.float32, parts: int = 1, gather: bool = True,
                 lanes: int = 1, independent: bool = False, launch: Optional[Callable] = None,
                 world: Optional[int] = None, rank: Optional[int] = None, row_block: int = 1):
        # world / rank: override the process group's (one process rehearsing rank `rank` of a
        # `world`-way split on one GPU; no exchange may then be requested)
        self.world = world or (dist.get_world_size(group) if dist.is_initialized() else 1)
        self.rank = rank if rank is not None else (dist.get_rank(group) if dist.is_initialized() else 0)
        if world is not None and gather:
            raise ValueError("a rehearsed split keeps its band (gather=False)")
        self.group = group
        self.width, self.height, self.parts = width, height, parts
        self.row_block = row_block
        if row_block > 1:   # block-cyclic band, one part, kept on its rank (bands may be unequal)
            if parts != 1 or gather:
                raise ValueError("block-cyclic bands are one part per lane and stay on their rank "
                                 "(parts=1, gather=False)")
            self.row0, self.rows, self.step = block_band_spec(self.rank, self.world, height, row_block)
            self.specs = [(self.row0, self.rows, self.step)]
        else:
            self.row0, self.rows, self.step = band_spec(self.rank, self.world, height)
            self.specs = [part_spec(self.rank, self.world, s, parts, height) for s in range(parts)]
        # render_band / launch receive row_block= only for block-cyclic bands
        self.block_kw = {"row_block": row_block} if row_block > 1 else {}
        self.rows_p = self.specs[0][1]
        self.render_band = render_band
        self.cuda = torch.device(device).type == "cuda"
        self.gather = gather and self.world > 1
        if lanes < 1 or (self.gather and lanes > 1):
            raise ValueError("lanes >= 1; frames in flight keep their bands on the ranks "
                             "(gather=False)")
        self.lanes, self.independent = lanes, independent
        self.channels, self.dtype = channels, dtype
        shape = (parts, self.rows_p, width, channels)
        self.bufs = None
        self.bands = None
        if not self.gather:
            # this rank's band per lane; part s renders band rows s, s + parts, ... in place
            self.bufs = [torch.zeros((self.rows, width, channels), dtype=dtype, device=device)
                         for _ in range(lanes)]
        else:
            self.bands = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(2)]
        self.part_streams = ([[torch.cuda.Stream(device=device) for _ in range(parts)]
                              for _ in range(lanes)]
                             if self.cuda and (parts > 1 or lanes > 1) else None)
        self.part_done = [[None] * parts for _ in range(lanes)]   # dependent lanes: frame events
        self.fresh = True   # the streams must first wait for the current stream's work
        self.assembly_stream = None
        self.gathered = None
        self.frame_buf = None
        if self.rank == 0 and self.gather:
            self.frame_buf = torch.empty((height, width, channels), dtype=dtype, device=device)
            self.gathered = [torch.empty((self.world,) + shape, dtype=dtype, device=device)
                             for _ in range(2)]
            if self.cuda:
                self.assembly_stream = torch.cuda.Stream(device=device)
        self.plan = None   # lean launches: per lane, per part (row0, rows, step, out, prev, pitch, stream)
        if (launch is not None and not self.gather and self.part_streams is not None
                and (lanes == 1 or independent)):
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
        self.pending = [None, None]     # gather that still reads bands[b]
        self.assembled = [None, None]   # rank 0: assembly that still reads gathered[b]
        self.prev = None                # rank 0: buffer index of the frame awaiting assembly
        self.k = 0

    # ---- helpers ---------------------------------------------------------------------------
    def part_rows(self, buf: torch.Tensor, s: int) -> torch.Tensor:
        """Part s's rows of a band buffer [rows, W, C] (band rows s, s + parts, ...)."""
        return buf.view(self.rows_p, self.parts, self.width, -1)[:, s]

    def last(self) -> torch.Tensor:
        """This rank's band buffer of the last frame enqueued (gather=False)."""
        return self.bufs[(self.k - 1) % self.lanes]

    def _part_buffers(self, s: int, band: torch.Tensor, prev: torch.Tensor):
        """(out, prev) of part s: its rows of the lane buffers, or its slot of the gather bands."""
        if not self.gather:
            return self.part_rows(band, s), self.part_rows(prev, s)
        return band[s], prev[s]

    def _render_parts(self, lane: int, band: torch.Tensor, prev: torch.Tensor, wait_work):
        """Enqueue every part of the next frame on `lane` (each first waits for `wait_work`, the
        gather that last read its buffer). Returns the parts' completion events (CUDA streams)."""
        if self.part_streams is None:
            if wait_work is not None:
                wait_work.wait()
            for s, (row0, rows, step) in enumerate(self.specs):
                self.render_band(row0, rows, step, *self._part_buffers(s, band, prev), **self.block_kw)
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
                if wait_work is not None:
                    wait_work.wait()
                if dep and self.part_done[prev_lane][s] is not None:
                    st.wait_event(self.part_done[prev_lane][s])   # the history rows of part s
                self.render_band(row0, rows, step, *self._part_buffers(s, band, prev), **self.block_kw)
                ev = st.record_event() if (dep or self.gather) else None
                self.part_done[lane][s] = ev
                events.append(ev)
        return events

    # ---- pipeline --------------------------------------------------------------------------
    def frame(self) -> Optional[torch.Tensor]:
        if self.plan is not None:   # lean launches from precomputed arguments
            lane = self.k % self.lanes
            self.k += 1
            if self.fresh:
                cur = torch.cuda.current_stream()
                for ln in self.part_streams:
                    for st in ln:
                        st.wait_stream(cur)
                self.fresh = False
            for args in self.plan[lane]:
                self.launch(*args, **self.block_kw)
            return self.bufs[lane]
        if not self.gather:   # one rank, or ranks that keep their bands: no exchange
            lane = self.k % self.lanes
            band, prev = self.bufs[lane], self.bufs[(self.k - 1) % self.lanes]
            self.k += 1
            self._render_parts(lane, band, prev, None)
            return band
        b = self.k % 2
        prev = self.bands[(self.k - 1) % 2]
        self.k += 1
        band = self.bands[b]
        wait_work, self.pending[b] = self.pending[b], None
        events = self._render_parts(0, band, prev, wait_work)
        cur = torch.cuda.current_stream() if self.cuda else None
        if events is not None:   # the gather (issued from the current stream) needs every part
            for e in events:
                cur.wait_event(e)
        if self.assembled[b] is not None:   # rank 0: the assembly that read gathered[b]
            cur.wait_event(self.assembled[b])
            self.assembled[b] = None
        glist = list(self.gathered[b].unbind(0)) if self.rank == 0 else None
        work = dist.gather(band, glist, dst=0, group=self.group, async_op=True)
        out = self._assemble_prev() if self.rank == 0 else None
        self.pending[b] = work
        if self.rank == 0:
            self.prev = b
        return out

    def _assemble_prev(self) -> Optional[torch.Tensor]:
        """Rank 0: re-interleave the previous frame's gathered parts into frame_buf once its
        gather is done (on the assembly stream when there is one). pending[b] is left for the
        next render into bands[b] to wait on."""
        if self.prev is None:
            return None
        b = self.prev
        self.prev = None
        work = self.pending[b]
        if self.assembly_stream is None:
            work.wait()
            return assemble_parts(self.gathered[b], self.frame_buf)
        with torch.cuda.stream(self.assembly_stream):
            work.wait()
            out = assemble_parts(self.gathered[b], self.frame_buf)
        self.assembled[b] = self.assembly_stream.record_event()
        return out

    def collect(self) -> Optional[torch.Tensor]:
        """Without the per-frame gather, after finish(): one gather of every rank's band of the
        last frame to rank 0, re-interleaved into the whole frame (returned on rank 0, None
        elsewhere); e.g. to display or check the last frame. Synchronous."""
        assert not self.gather, "collect() is for gather=False tilers"
        band = self.last().contiguous()
        if self.world == 1:
            return band
        if self.row_block == 1:
            glist = ([torch.empty_like(band) for _ in range(self.world)] if self.rank == 0 else None)
            dist.gather(band, glist, dst=0, group=self.group)
            return assemble_cyclic(torch.stack(glist)) if self.rank == 0 else None
        # block-cyclic bands may differ by one block: gather them padded to the largest
        specs = [block_band_spec(r, self.world, self.height, self.row_block) for r in range(self.world)]
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

    def finish(self) -> Optional[torch.Tensor]:
        cur = torch.cuda.current_stream() if self.cuda else None
        if not self.gather:
            for ln in self.part_streams or ():
                for st in ln:
                    cur.wait_stream(st)
            self.fresh = True
            return self.last()
        out = self._assemble_prev() if self.rank == 0 else None
        for i, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[i] = None
        for ln in self.part_streams or ():
            for st in ln:
                cur.wait_stream(st)
        if self.assembly_stream is not None:
            cur.wait_stream(self.assembly_stream)
        self.fresh = True
        return out
