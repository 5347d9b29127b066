"""Config 4 (BASELINE configs[3]: 3840x2160 1 spp of the config-3 room, the frame split across N GPUs in
8-row bands) one rank's share at a time, on one MI355X: the frame time of rank 0's bands for N = 1, 2, 4, 8,
timed like bench.py's steps (warmup, K frames between two synchronisations).  With the bands interleaved
every rank's share is the same work, so N x (the N = 1 time / the share's time) is the strong-scaling
factor the rendering allows before the accumulator gather (which overlaps the next frame's rendering in
bench.py: the core stream does not wait for it).  One JSON line per N on stdout.
"""
from __future__ import annotations

import argparse
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402  (one HIP runtime in the process)

from lighthouse2_amd import scene  # noqa: E402
from lighthouse2_amd.core import RenderCore  # noqa: E402
from lighthouse2_amd.parallel import BAND  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--room-tris", type=int, default=1_000_000)
    ap.add_argument("--setting", action="append", default=[], help="name=value core setting")
    args = ap.parse_args()
    W4, H4 = 3840, 2160
    sc = scene.room_scene(args.room_tris, W4, H4)
    base = None
    for n in [int(x) for x in args.ranks.split(",")]:
        core = RenderCore(device=0)
        core.setting("maxPathLength", 4)
        for kv in args.setting:
            core.setting(kv.split("=")[0], float(kv.split("=")[1]))
        sc.load_into(core)
        core.set_target(W4, H4, 1)
        core.set_tile_bands(0, n, BAND)
        for i in range(args.warmup):
            sc.render_frame(core, converge=1 if i == 0 else 0)   # a converging still camera, as bench.py
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.frames):
            sc.render_frame(core, converge=0)
        core.sync()
        ms = (time.perf_counter() - t0) / args.frames * 1e3
        counts = core.ray_counts()
        base = base or ms
        print(json.dumps({"ranks": n, "rows": core.tile_rows(), "paths": int(counts[0]), "ms_per_frame": round(ms, 4),
                          "render_scaling": round(base / ms, 3),
                          "primary_plus_bounce1": int(counts[0]) + int(counts[1])}), flush=True)
        core.close()


if __name__ == "__main__":
    main()
