"""The fixed cost of config 4's per-frame accumulator gather at N ranks, measured on one MI355X:
  pack    the core's k_pack_rows of one rank's owned rows into its send tile (every rank, on its own GPU);
  copy    the tile's bytes copied device-to-device on this GPU: HBM-local, so a floor; the xGMI leg is modelled at
          the stated 153 GB/s per link, the N - 1 tiles arriving at rank 0 over N - 1 links in parallel;
  unpack  rank 0's assembly of the frame from the N stacked tiles (parallel.TileGather: one index_select of the
          whole frame, what bench.py's config4 runs), and the row scatter of the other ranks' rows only (k_unpack_rows'
          work: 16 B read + 16 B written per pixel of N - 1 tiles) timed as an index_copy_.
All on the GPU with HIP events on the stream each step runs on; the frames are rendered once first, so the tiles hold
real rows.  One JSON line on stdout.
"""
from __future__ import annotations

import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lighthouse2_amd import scene  # noqa: E402
from lighthouse2_amd.core import RenderCore  # noqa: E402
from lighthouse2_amd.parallel import BAND, band_rows, frame_row_sources  # noqa: E402

XGMI_LINK_GBS = 153.0   # per link, the stated MI355X figure (7 links per GPU)


def timed(fn, stream, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        fn()
        s.record(stream)
        for _ in range(iters):
            fn()
        e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--room-tris", type=int, default=1_000_000)
    args = ap.parse_args()
    N, W, H = args.ranks, 3840, 2160
    dev = torch.device("cuda", 0)
    sc = scene.room_scene(args.room_tris, W, H)
    core = RenderCore(device=0)
    core.setting("maxPathLength", 4)
    sc.load_into(core)
    core.set_target(W, H, 1)
    core.set_tile_bands(1, N, BAND)          # a rank other than 0: its rows go over a link
    sc.render_frame(core, converge=1)
    core.sync()
    rows = core.tile_rows()
    maxrows = max(len(band_rows(r, N, H)) for r in range(N))
    send = torch.empty((maxrows, W, 4), dtype=torch.float32, device=dev)
    core_stream = torch.cuda.ExternalStream(core.stream_ptr(), device=dev)
    pack_ms = timed(lambda: core.pack_tile(send.data_ptr(), order_torch=False), core_stream, args.iters)
    tile_bytes = rows * W * 16
    recv = torch.empty((N * maxrows, W, 4), dtype=torch.float32, device=dev)
    recv.view(N, maxrows, W, 4)[:] = send
    st = torch.cuda.current_stream()
    copy_ms = timed(lambda: recv[maxrows:2 * maxrows].copy_(send), st, args.iters)
    frame = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
    src = torch.as_tensor(frame_row_sources(N, H), device=dev)
    assemble_ms = timed(lambda: torch.index_select(recv, 0, src, out=frame), st, args.iters)
    others = np.concatenate([band_rows(r, N, H) for r in range(1, N)])
    dst_rows = torch.as_tensor(others, device=dev)
    src_rows = torch.as_tensor(frame_row_sources(N, H)[others], device=dev)
    scatter_ms = timed(lambda: frame.index_copy_(0, dst_rows, recv.index_select(0, src_rows)), st, args.iters)
    xgmi_ms = tile_bytes / (XGMI_LINK_GBS * 1e9) * 1e3
    core.close()
    print(json.dumps({"ranks": N, "frame": [W, H], "tile_rows": rows, "tile_MB": round(tile_bytes / 1e6, 2),
                      "rank0_receives_MB": round((N - 1) * tile_bytes / 1e6, 1),
                      "pack_ms": round(pack_ms, 4), "hbm_copy_ms_per_tile": round(copy_ms, 4),
                      "xgmi_model_ms": round(xgmi_ms, 4), "xgmi_model": f"{round(tile_bytes / 1e6, 2)} MB per tile / "
                      f"{XGMI_LINK_GBS} GB/s per link, the {N - 1} tiles over {N - 1} links in parallel",
                      "assemble_index_select_ms": round(assemble_ms, 4), "scatter_other_rows_ms": round(scatter_ms, 4),
                      "fixed_cost_model_ms": round(pack_ms + xgmi_ms + assemble_ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
