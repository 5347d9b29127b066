"""Multi-GPU frame partition: one process per GPU, each rendering a set of row bands
of the frame, then one accumulator gather to rank 0 per frame.

The path tracer's work items are pixels: a path only ever touches its own pixel
(pathtracer.h:79-80, connections.h:31-33) and its random numbers depend only on the global pixel
index, sample index and R0 (camera.h:50-70, pathtracer.h:159,174-176).  A partition is therefore
exact as long as every rank uses global pixel coordinates, which the core does (SetTileBands).
Rows are dealt in bands of BAND rows round-robin over ranks so that every rank gets a similar mix
of sky and geometry.  The only collective is the gather of the finished accumulator rows
(torch.distributed: RCCL over xGMI with backend "nccl", gloo on CPU for the tests).

`TileGather` holds every buffer of the exchange, allocated once per frame size: the (padded) send
tile the core packs its rows into, rank 0's receive block and frame, and the row map that turns
the received blocks into the frame with one index_select.  A frame then costs the pack, one
collective and (rank 0) one gather kernel, with no allocation and no host-to-device index upload.
The in-process multi-device mode of the core itself (setting "deviceCount", csrc/multidevice.cpp) is
the same partition with xGMI peer copies instead of a collective.
"""
from __future__ import annotations

import numpy as np

BAND = 8


def band_rows(rank: int, nranks: int, height: int, band: int = BAND) -> np.ndarray:
    """Global frame rows owned by `rank`, in the core's local (packing) order."""
    rows = []
    y = rank * band
    while y < height:
        rows.extend(range(y, min(y + band, height)))
        y += nranks * band
    return np.asarray(rows, dtype=np.int64)


def frame_row_sources(nranks: int, height: int, band: int = BAND) -> np.ndarray:
    """For every frame row, its row in the stacked receive block (rank r's rows start at r * maxrows)."""
    sizes = [len(band_rows(r, nranks, height, band)) for r in range(nranks)]
    maxrows = max(sizes)
    src = np.empty(height, np.int64)
    for r in range(nranks):
        src[band_rows(r, nranks, height, band)] = r * maxrows + np.arange(sizes[r])
    return src


def assemble(tiles, nranks: int, height: int, band: int = BAND):
    """Host-side scatter of the per-rank row blocks (rows, width, 4) into the full frame (tests)."""
    width = tiles[0].shape[1]
    out = np.empty((height, width, 4), dtype=tiles[0].dtype)   # the bands cover every row
    for r, t in enumerate(tiles):
        out[band_rows(r, nranks, height, band)] = t
    return out


class TileGather:
    """The frame exchange of one rank: `send` is the tile the core packs its owned rows into (padded to
    the largest rank's row count: the collective needs equal shapes), `gather()` collects every rank's
    tile on rank 0 and returns the assembled frame there (None elsewhere)."""

    def __init__(self, rank: int, nranks: int, width: int, height: int, device, band: int = BAND):
        import torch
        self.rank, self.nranks, self.width, self.height, self.band = rank, nranks, width, height, band
        self.rows = len(band_rows(rank, nranks, height, band))
        self.maxrows = max(len(band_rows(r, nranks, height, band)) for r in range(nranks))
        self.send = torch.empty((self.maxrows, width, 4), dtype=torch.float32, device=device)
        self.recv = self.recv_list = self.frame = self.src = None
        if rank == 0 and nranks > 1:
            self.recv = torch.empty((nranks * self.maxrows, width, 4), dtype=torch.float32, device=device)
            self.recv_list = list(self.recv.view(nranks, self.maxrows, width, 4).unbind(0))
            self.frame = torch.empty((height, width, 4), dtype=torch.float32, device=device)
            self.src = torch.as_tensor(frame_row_sources(nranks, height, band), device=device)

    @property
    def tile(self):
        """The owned rows, in the core's packing order (a view of `send`)."""
        return self.send[: self.rows]

    def gather(self):
        import torch
        import torch.distributed as dist
        if self.nranks == 1:
            return self.send                 # one rank owns every row, in frame order
        dist.gather(self.send, self.recv_list if self.rank == 0 else None, dst=0)
        if self.rank != 0:
            return None
        torch.index_select(self.recv, 0, self.src, out=self.frame)
        return self.frame


def gather_tiles(tile, rank: int, nranks: int, height: int, band: int = BAND):
    """One-off gather of every rank's packed rows to rank 0 (tests; frame loops use TileGather)."""
    g = TileGather(rank, nranks, tile.shape[1], height, tile.device, band)
    g.tile.copy_(tile)
    return g.gather()
