"""Row-tile partitioning across ranks and the gather that assembles a frame.

Rank r of N renders the rows y = r, r+N, r+2N, ... (interleaved single rows balance the
sky-vs-ground cost of the reference scene). Every RNG stream is keyed by the global
(pixel, sample), so the assembled frame is bitwise independent of N. The exchange is one
gather of the packed per-rank tiles to rank 0 (RCCL over xGMI on GPUs, gloo on CPU) followed
by one strided copy that de-interleaves them.
"""
import torch
import torch.distributed as dist

from .render import make_params


def rank_rows(height, world, rank):
    """(row_offset, row_stride, num_rows) of rank `rank`; equal tiles need height % world == 0."""
    if height % world:
        raise ValueError(f"height {height} is not divisible by {world} ranks")
    return rank, world, height // world


def rank_params(width, height, spp, world, rank, **kw):
    off, stride, rows = rank_rows(height, world, rank)
    return make_params(width, height, spp, row_offset=off, row_stride=stride, num_rows=rows, **kw)


class FrameGather:
    """Gathers packed (rows, W, 3) tiles into the (H, W, 3) frame on rank 0."""

    def __init__(self, tile, world, rank, group=None):
        self.world, self.rank, self.group = world, rank, group
        self.rows, self.width = tile.shape[0], tile.shape[1]
        # rank 0 gathers the tiles into one (world, rows, W, 3) buffer (each part a contiguous
        # slice of it), then de-interleaves it into the frame with ONE strided copy
        self.gathered = torch.empty((world, self.rows, self.width, 3), dtype=tile.dtype, device=tile.device) \
            if rank == 0 and world > 1 else None
        self.parts = list(self.gathered.unbind(0)) if self.gathered is not None else None
        self.frame = torch.empty((self.rows * world, self.width, 3), dtype=tile.dtype, device=tile.device) \
            if rank == 0 and world > 1 else None

    def __call__(self, tile):
        if self.world == 1:  # the one tile is the frame
            return tile
        dist.gather(tile, gather_list=self.parts, dst=0, group=self.group)
        if self.rank == 0:
            # frame row y = i*world + r  <-  tile r row i
            self.frame.view(self.rows, self.world, self.width, 3).copy_(self.gathered.transpose(0, 1))
        return self.frame
