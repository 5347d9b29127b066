"""Multi-GPU frame partition: one process per GPU, each rendering a set of row bands
of the frame, then one accumulator gather to rank 0 per frame.

The path tracer's work items are pixels: a path only ever touches its own pixel
(pathtracer.h:79-80, connections.h:31-33) and its random numbers depend only on the global pixel
index, sample index and R0 (camera.h:50-70, pathtracer.h:159,174-176).  A partition is therefore
exact as long as every rank uses global pixel coordinates, which the core does (SetTileBands).
Rows are dealt in bands of BAND rows round-robin over ranks so that every rank gets a similar mix
of sky and geometry.  The only collective is the gather of the finished accumulator rows
(torch.distributed: RCCL over xGMI with backend "nccl", gloo on CPU for the tests).
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


def assemble(tiles, nranks: int, height: int, band: int = BAND, xp=np):
    """Rank 0: scatter the gathered per-rank row blocks (rows, width, 4) into the full frame."""
    width = tiles[0].shape[1]
    # the ranks' bands partition the rows, so every row of the frame is written: no zero fill
    out = xp.empty((height, width, 4), dtype=tiles[0].dtype) if xp is np else None
    if out is None:  # torch
        import torch
        out = torch.empty((height, width, 4), dtype=tiles[0].dtype, device=tiles[0].device)
        for r, t in enumerate(tiles):
            idx = torch.as_tensor(band_rows(r, nranks, height, band), device=t.device)
            out.index_copy_(0, idx, t)
        return out
    for r, t in enumerate(tiles):
        out[band_rows(r, nranks, height, band)] = t
    return out


def gather_tiles(tile, rank: int, nranks: int, height: int, band: int = BAND):
    """torch.distributed gather of every rank's packed rows to rank 0; returns the frame on rank 0."""
    import torch
    import torch.distributed as dist
    sizes = [len(band_rows(r, nranks, height, band)) for r in range(nranks)]
    if nranks == 1:
        return tile                      # one rank owns every row, in frame order
    maxrows = max(sizes)
    width = tile.shape[1]
    send = tile
    if tile.shape[0] < maxrows:   # gather needs equal shapes: pad the short ranks
        send = torch.zeros((maxrows, width, 4), dtype=tile.dtype, device=tile.device)
        send[: tile.shape[0]] = tile
    bufs = [torch.empty_like(send) for _ in range(nranks)] if rank == 0 else None
    dist.gather(send, bufs, dst=0)
    if rank != 0:
        return None
    return assemble([b[: sizes[r]] for r, b in enumerate(bufs)], nranks, height, band, xp=torch)
