"""Framebuffer tiling across the GPUs of one node.

The per-pixel program has no halo and no inter-ray exchange, so a frame splits into row bands,
one per rank (one process per GPU). Bands are cyclic — rank r owns rows r, r+N, r+2N, ... — so
every rank gets the same mix of cheap sky rows and expensive geometry rows. Each rank renders its
band into HBM; the only exchange is one gather of the bands to rank 0 per frame (RCCL over xGMI
with the "nccl" backend; gloo on CPU for tests), after which rank 0 re-interleaves the bands into
the frame. The volume is replicated once per GPU (broadcast_volume).

Within a rank the band is rendered as P interleaved parts on P HIP streams (default P = 1; the
bench uses 2): global part q = s*N + r owns frame rows q, q + N*P, q + 2*N*P, ... . One launch's
last dispatch round leaves wave slots idle while its final waves finish; a second stream's launch
fills them, so consecutive frames' parts overlap their tails (measured: C3 0.241 -> 0.220 ms per
frame with P = 2, scripts/streams_exp.py). Ordering uses events only: a part stream waits for the
gather that last read its buffer, the gather waits for every part of its frame — a part never
waits for another part, so the overlap is real.

With one rank and P > 1 parts, every part renders straight into its rows of the frame buffer
(a row-strided view; the renderer's row pitch, ABI v4) and filters them in place against the same
rows, which hold the previous frame: no band buffers, no assembly copy (it cost ≈4 % of a C3
frame as two strided copy kernels per frame).

With several ranks the frame is either gathered to rank 0 every frame (gather=True: the display
of one whole frame on one GPU) or kept distributed (gather=False, bench.py's default for N > 1):
the per-pixel program has no exchange step, so each rank then renders and filters its band in
place exactly as a single rank renders its frame, and collect() gathers the bands once when the
whole frame is wanted (SURVEY §8e's per-frame gather is output delivery, not part of the path: at
weak scaling every rank's 8.3 MB RGBA8 band would cross xGMI into rank 0 per 0.06 ms frame).
FrameTiler double-buffers the band (gather=True) so that the gather of frame k overlaps the render
of frame k+1. Bands are RGBA8 words when the renderer runs the fused temporal filter + RGB8 store
(the reference's stored frame format, main.cpp:363-393): 4 B per pixel on the wire instead of 16.
The temporal history is part-local (each part blends its own rows, on its own stream), so it adds
no exchange and no cross-stream dependency; the previous frame's part buffer IS the history.
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
    """Renders a sequence of frames across `world` ranks, `parts` streams per rank.

    render_band(row0, rows, row_step, out, prev) must enqueue the render of one part into `out`
    ([rows, W, channels] of `dtype` on `device`; possibly a row-strided view, see row_pitch) on
    the CURRENT stream (the HIP kernel through the C-ABI, or the oracle in CPU tests); `prev` holds
    that part's rows of the previous frame (the temporal history; zeros before the first frame;
    it is `out` itself with one buffer: each pixel is read before it is written).
    frame() renders the next frame; with one rank, or with gather=False, it returns this rank's
    band of it (the whole frame with one rank; for parts > 1 each part renders into its rows of it
    directly, in place); with several ranks and gather=True the gather is issued asynchronously
    and rank 0 returns the PREVIOUS frame, assembled on `self.assembly_stream` (None on the first
    call and on other ranks), so the gather of frame k overlaps the render of frame k+1. finish()
    drains the pipeline and returns the last frame (band) on rank 0; collect() (gather=False)
    assembles the last frame on rank 0 with one gather. A returned frame is valid until the next
    frame() call; synchronise the device before reading it.
    """

    def __init__(self, width: int, height: int, render_band: Callable, device, group=None,
                 channels: int = 4, dtype=torch.float32, parts: int = 1, gather: bool = True):
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.group = group
        self.width, self.height, self.parts = width, height, parts
        self.row0, self.rows, self.step = band_spec(self.rank, self.world, height)
        self.specs = [part_spec(self.rank, self.world, s, parts, height) for s in range(parts)]
        self.rows_p = self.specs[0][1]
        self.render_band = render_band
        self.cuda = torch.device(device).type == "cuda"
        self.gather = gather and self.world > 1
        self.channels, self.dtype = channels, dtype
        shape = (parts, self.rows_p, width, channels)
        nbuf = 2 if self.gather else 1
        # no per-frame gather, several parts: the parts render into (and filter in place) this
        # rank's band itself (the whole frame with one rank)
        self.direct = not self.gather and parts > 1
        self.frame_buf = None
        if self.direct:
            self.frame_buf = torch.zeros((self.rows, width, channels), dtype=dtype, device=device)
            self.bands = [self.frame_buf.view(shape)]   # same storage (bench's counted launch)
        else:
            self.bands = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(nbuf)]
        self.part_streams = ([torch.cuda.Stream(device=device) for _ in range(parts)]
                             if self.cuda and parts > 1 else None)
        self.assembly_stream = None
        self.gathered = None
        if self.rank == 0 and self.gather:
            self.frame_buf = torch.empty((height, width, channels), dtype=dtype, device=device)
        if self.rank == 0 and self.gather:
            self.gathered = [torch.empty((self.world,) + shape, dtype=dtype, device=device)
                             for _ in range(nbuf)]
            if self.cuda:
                self.assembly_stream = torch.cuda.Stream(device=device)
        self.pending = [None] * nbuf    # gather that still reads bands[b]
        self.assembled = [None] * nbuf  # rank 0: assembly that still reads gathered[b] / bands[b]
        self.prev = None                # rank 0: buffer index of the frame awaiting assembly
        self.k = 0

    # ---- helpers ---------------------------------------------------------------------------
    def _part_buffers(self, s: int, band: torch.Tensor, prev: torch.Tensor):
        """(out, prev) of part s: its rows of the frame (in place) in direct mode, else its slot
        of the band buffers."""
        if self.direct:
            rows = self._frame_rows(s)
            return rows, rows
        return band[s], prev[s]

    def _render_parts(self, band: torch.Tensor, prev: torch.Tensor, wait_work):
        """Enqueue every part (each waits for `wait_work`, the gather that last read its buffer).
        Returns the events that mark the parts' completion (CUDA, parts > 1)."""
        if self.part_streams is None:
            if wait_work is not None:
                wait_work.wait()
            for s, (row0, rows, step) in enumerate(self.specs):
                self.render_band(row0, rows, step, *self._part_buffers(s, band, prev))
            return None
        events = []
        for s, (row0, rows, step) in enumerate(self.specs):
            st = self.part_streams[s]
            with torch.cuda.stream(st):
                if wait_work is not None:
                    wait_work.wait()
                self.render_band(row0, rows, step, *self._part_buffers(s, band, prev))
                events.append(st.record_event())
        return events

    def _frame_rows(self, s: int) -> torch.Tensor:
        """frame_buf rows of this rank's part s (direct mode: frame_buf is the rank's band, the
        whole frame with one rank): band rows s, s + parts, ..."""
        return self.frame_buf.view(self.rows_p, self.parts, self.width, -1)[:, s]

    # ---- pipeline --------------------------------------------------------------------------
    def frame(self) -> Optional[torch.Tensor]:
        nb = len(self.bands)
        b = self.k % nb
        prev = self.bands[(self.k - 1) % nb]
        self.k += 1
        band = self.bands[b]
        if not self.gather:   # one rank, or ranks that keep their bands: no exchange
            self._render_parts(band, prev, None)
            return band[0] if self.parts == 1 else self.frame_buf
        wait_work, self.pending[b] = self.pending[b], None
        events = self._render_parts(band, prev, wait_work)
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
        """Without the per-frame gather, after finish(): one gather of every rank's current band to
        rank 0, re-interleaved into the whole frame (returned on rank 0, None elsewhere); e.g. to
        display or check the last frame. Synchronous."""
        assert not self.gather, "collect() is for gather=False tilers"
        band = (self.frame_buf if self.direct else self.bands[0][0]).contiguous()
        if self.world == 1:
            return band
        glist = ([torch.empty_like(band) for _ in range(self.world)] if self.rank == 0 else None)
        dist.gather(band, glist, dst=0, group=self.group)
        return assemble_cyclic(torch.stack(glist)) if self.rank == 0 else None

    def finish(self) -> Optional[torch.Tensor]:
        if not self.gather:
            if self.part_streams is not None:
                cur = torch.cuda.current_stream()
                for st in self.part_streams:
                    cur.wait_stream(st)
            return self.bands[0][0] if self.parts == 1 else self.frame_buf
        out = self._assemble_prev() if self.rank == 0 else None
        for i, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[i] = None
        cur = torch.cuda.current_stream() if self.cuda else None
        for st in self.part_streams or ():
            cur.wait_stream(st)
        if self.assembly_stream is not None:
            cur.wait_stream(self.assembly_stream)
        return out
