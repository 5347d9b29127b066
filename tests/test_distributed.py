"""Multi-rank frame partition on CPU: world_size 2 with the gloo backend.

Each rank renders only its 8-row bands (the partition bench.py uses on N GPUs), packs them and
gathers to rank 0 with lighthouse2_amd.parallel.gather_tiles (the same code path that runs over
RCCL on MI355X).  Rank 0 must reassemble exactly the single-process full frame.  The per-rank
renderer here is the CPU oracle: the test covers the partition + collective logic, while
tests/test_gpu_parity.py::test_band_partition_matches_full_frame covers the HIP side."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lighthouse2_amd import parallel, scene
from oracle.oracle import Oracle

W, H = 64, 44     # 44 rows: the last band is partial


def _scene():
    return scene.room_scene(6000, W, H)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = _scene()
        o = Oracle(threads=2)
        sc.load_into(o)
        o.set_target(W, H, 1)
        o.set_tile_bands(rank, world, parallel.BAND)
        sc.render_frame(o)
        rows = parallel.band_rows(rank, world, H)
        tile = torch.from_numpy(np.ascontiguousarray(o.accumulator()[rows]))
        frame = parallel.gather_tiles(tile, rank, world, H)
        if rank == 0:
            q.put(frame.numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_band_partition_gather_equals_full_frame(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sc = _scene()
    o = Oracle(threads=4)
    sc.load_into(o)
    o.set_target(W, H, 1)
    sc.render_frame(o)
    full = o.accumulator()
    assert np.array_equal(frame, full)


def test_band_rows_partition_the_frame():
    for world in (1, 2, 3, 8):
        for h in (1, 7, 8, 44, 1080, 2160):
            rows = np.concatenate([parallel.band_rows(r, world, h) for r in range(world)])
            assert np.array_equal(np.sort(rows), np.arange(h))
