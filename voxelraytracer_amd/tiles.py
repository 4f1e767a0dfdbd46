"""Framebuffer tiling across the GPUs of one node.

The per-pixel program has no halo and no inter-ray exchange, so a frame splits into row bands,
one per rank (one process per GPU). Bands are cyclic — rank r owns rows r, r+N, r+2N, ... — so
every rank gets the same mix of cheap sky rows and expensive geometry rows. Each rank renders its
band into HBM; the only exchange is one gather of the RGBA bands to rank 0 per frame (RCCL over
xGMI with the "nccl" backend; gloo on CPU for tests), after which rank 0 re-interleaves the bands
into the frame. The volume is replicated once per GPU (broadcast_volume).

FrameTiler double-buffers the band so that, over a sequence of frames, the gather of frame k
overlaps the render of frame k+1 on the compute stream. Bands are RGBA8 words when the renderer
runs the fused temporal filter + RGB8 store (the reference's stored frame format, main.cpp:363-393):
4 B per pixel on the wire instead of 16. The temporal history is band-local (each rank blends its
own rows), so it adds no exchange; the previous frame's band buffer IS the history.
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


def assemble_cyclic(bands: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bands[world, rows, W, C] (rank-major) -> frame[rows*world, W, C] with frame row i*world+r
    = bands[r, i]."""
    world, rows, w, c = bands.shape
    if out is None:
        out = torch.empty((rows * world, w, c), dtype=bands.dtype, device=bands.device)
    out.view(rows, world, w, c).copy_(bands.permute(1, 0, 2, 3))
    return out


def broadcast_volume(vox: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    """Replicate the N^3 volume (uint8 tensor on this rank's device) from `src` to every rank."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(vox, src, group=group)
    return vox


class FrameTiler:
    """Renders a sequence of frames across `world` ranks.

    render_band(row0, rows, row_step, out, prev) must enqueue the band render into `out`
    ([rows, W, channels] of `dtype` on `device`) on the current stream (the HIP kernel through the
    C-ABI, or the oracle in CPU tests); `prev` holds this rank's band of the previous frame (the
    temporal history; zeros before the first frame; it is `out` itself with one buffer).
    frame() renders the next frame and issues its gather asynchronously; on rank 0 it returns the
    PREVIOUS frame, assembled (None on the first call and on other ranks), so the gather of frame
    k overlaps the render of frame k+1 on every rank. Rank 0 re-interleaves on a side stream
    (returned frames are ordered on `self.assembly_stream`). finish() drains the pipeline and
    returns the last frame on rank 0.
    """

    def __init__(self, width: int, height: int, render_band: Callable, device, group=None,
                 channels: int = 4, dtype=torch.float32):
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.group = group
        self.width, self.height = width, height
        self.row0, self.rows, self.step = band_spec(self.rank, self.world, height)
        self.render_band = render_band
        shape = (self.rows, width, channels)
        nbuf = 2 if self.world > 1 else 1
        self.bands = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(nbuf)]
        self.assembly_stream = None
        if self.rank == 0 and self.world > 1 and torch.device(device).type == "cuda":
            self.assembly_stream = torch.cuda.Stream(device=device)
        self.gathered = None
        self.frame_buf = None
        if self.rank == 0 and self.world > 1:
            self.gathered = [torch.empty((self.world,) + shape, dtype=dtype, device=device)
                             for _ in range(nbuf)]
            self.frame_buf = torch.empty((height, width, channels), dtype=dtype, device=device)
        self.pending = [None] * nbuf   # gather that still reads bands[b]
        self.assembled = [None] * nbuf  # rank 0: assembly that still reads gathered[b]
        self.prev = None               # rank 0: buffer index of the frame awaiting assembly
        self.k = 0

    def _assemble_prev(self) -> Optional[torch.Tensor]:
        if self.prev is None:
            return None
        b = self.prev
        self.prev = None
        if self.assembly_stream is not None:
            with torch.cuda.stream(self.assembly_stream):
                self.pending[b].wait()          # the side stream waits for the gather
                self.pending[b] = None
                out = assemble_cyclic(self.gathered[b], self.frame_buf)
            self.assembled[b] = self.assembly_stream.record_event()
            return out
        self.pending[b].wait()
        self.pending[b] = None
        return assemble_cyclic(self.gathered[b], self.frame_buf)

    def frame(self) -> Optional[torch.Tensor]:
        if self.world == 1:
            self.render_band(self.row0, self.rows, self.step, self.bands[0], self.bands[0])
            return self.bands[0]
        b = self.k % len(self.bands)
        prev = self.bands[(self.k - 1) % len(self.bands)]
        self.k += 1
        if self.pending[b] is not None:   # the gather that last read this buffer must be done
            self.pending[b].wait()
            self.pending[b] = None
        band = self.bands[b]
        self.render_band(self.row0, self.rows, self.step, band, prev)
        if self.assembled[b] is not None:   # rank 0: the assembly that read gathered[b]
            torch.cuda.current_stream().wait_event(self.assembled[b])
            self.assembled[b] = None
        glist = list(self.gathered[b].unbind(0)) if self.rank == 0 else None
        work = dist.gather(band, glist, dst=0, group=self.group, async_op=True)
        out = self._assemble_prev() if self.rank == 0 else None
        self.pending[b] = work
        if self.rank == 0:
            self.prev = b
        return out

    def finish(self) -> Optional[torch.Tensor]:
        if self.world == 1:
            return self.bands[0]
        out = self._assemble_prev() if self.rank == 0 else None
        for i, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[i] = None
        return out
