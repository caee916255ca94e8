"""Row-tile partitioning across ranks and the gather that assembles a frame.

Rank r of N renders the rows y = r, r+N, r+2N, ... (interleaved single rows balance the
sky-vs-ground cost of the reference scene); when N does not divide the height the first
H mod N ranks hold one row more (ragged tiles). Every RNG stream is keyed by the global
(pixel, sample), so the assembled frame is bitwise independent of N. The exchange is one
gather of the per-rank tiles to rank 0 (RCCL over xGMI on GPUs, gloo on CPU), each tile in a
slot of the largest tile's size, followed by one strided copy per slot height that
de-interleaves them. f32 tiles (12 B per pixel) or u8 tiles after the gamma epilogue (3 B).
"""
import torch
import torch.distributed as dist

from .render import make_params


def rank_rows(height, world, rank):
    """(row_offset, row_stride, num_rows) of rank `rank`: rows rank, rank + world, ... below height."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside a world of {world}")
    return rank, world, max(0, (height - rank + world - 1) // world)


def rank_params(width, height, spp, world, rank, **kw):
    off, stride, rows = rank_rows(height, world, rank)
    if rows == 0:
        raise ValueError(f"rank {rank} of {world} has no rows of a {height}-row frame")
    return make_params(width, height, spp, row_offset=off, row_stride=stride, num_rows=rows, **kw)


class FrameGather:
    """Gathers packed (rows_r, W, 3) tiles into the (H, W, 3) frame on rank 0 (f32 or u8)."""

    def __init__(self, tile, world, rank, height=None, group=None):
        self.world, self.rank, self.group = world, rank, group
        self.rows, self.width = tile.shape[0], tile.shape[1]
        self.height = height if height is not None else self.rows * world
        self.rows_max = rank_rows(self.height, world, 0)[2]
        if self.rows != rank_rows(self.height, world, rank)[2]:
            raise ValueError(f"rank {rank}: a tile of {self.rows} rows, expected "
                             f"{rank_rows(self.height, world, rank)[2]} of a {self.height}-row frame")
        self.ragged = self.height % world != 0
        # every rank sends a slot of rows_max rows (its own rows first); rank 0 gathers them into
        # one (world, rows_max, W, 3) buffer and de-interleaves it into the frame
        self.send = torch.empty((self.rows_max, self.width, 3), dtype=tile.dtype, device=tile.device) \
            if self.ragged and world > 1 else None
        self.gathered = torch.empty((world, self.rows_max, self.width, 3), dtype=tile.dtype, device=tile.device) \
            if rank == 0 and world > 1 else None
        self.parts = list(self.gathered.unbind(0)) if self.gathered is not None else None
        self.frame = torch.empty((self.height, self.width, 3), dtype=tile.dtype, device=tile.device) \
            if rank == 0 and world > 1 else None

    def __call__(self, tile):
        if self.world == 1:  # the one tile is the frame
            return tile
        src = tile
        if self.ragged:
            self.send[:self.rows].copy_(tile)
            src = self.send
        dist.gather(src, gather_list=self.parts, dst=0, group=self.group)
        if self.rank == 0:
            full = self.height // self.world  # rows every rank holds
            # frame row y = i*world + r  <-  tile r row i, for the rows every rank holds ...
            self.frame[:full * self.world].view(full, self.world, self.width, 3).copy_(
                self.gathered[:, :full].transpose(0, 1))
            # ... and the last, partial row group (ranks r < H mod world hold one row more)
            extra = self.height - full * self.world
            if extra:
                self.frame[full * self.world:].copy_(self.gathered[:extra, full])
        return self.frame
