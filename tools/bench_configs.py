"""Measure the other single-GPU BASELINE.json configurations on one MI355X.

  config3: full wavefront path trace, maxPathLength 4, 1M-triangle procedural room (walls, columns,
           smooth spheres, clutter; 70 % diffuse, 20 % specular, 10 % glass; two emissive quads),
           1080p 1 spp.
  config5: 100 distinct 100k-triangle meshes (10M triangles), one instance each on a 10 x 10 grid,
           new seeded rotations of every instance each frame (SetInstance x 100 + UpdateToplevel),
           1080p 8 spp.

Reported per config: Mrays/s = (primary + bounce-1 rays) / frame time (the bench.py metric), all
extension rays per frame, shadow rays, the CoreStats trace/shade times, and the host setup time.
One JSON line per config on stdout.  Parity of both configurations, at reduced size, is covered by
tests/test_gpu_parity.py (room scene, instanced scene with per-frame instance updates).
"""
from __future__ import annotations

import argparse
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402,F401  (one HIP runtime in the process)

from lighthouse2_amd import scene  # noqa: E402
from lighthouse2_amd.core import RenderCore  # noqa: E402


def measure(core, sc, frames, warmup, per_frame=None, converge_each=False):
    """frames timed like bench.py's step loop: one synchronize before and after the K frames (the host
    queues frame i+1 while the GPU renders frame i); the per-frame-synchronised time (the host's launch
    latency exposed every frame) is reported beside it"""
    def frame(i):
        if per_frame:
            per_frame(i)
        sc.render_frame(core, converge=1 if converge_each else (1 if i == 0 else 0))
    for i in range(warmup):
        frame(i)
    core.sync()
    counts = core.ray_counts()
    t0 = time.perf_counter()
    for i in range(frames):
        frame(warmup + i)
    core.sync()
    el = (time.perf_counter() - t0) / frames
    st = core.stats()
    t0 = time.perf_counter()
    for i in range(frames):
        frame(warmup + frames + i)
        core.sync()
    el_sync = (time.perf_counter() - t0) / frames
    return {"ms_per_frame": round(el * 1e3, 3),
            "Mrays_s": round((int(counts[0]) + int(counts[1])) / el / 1e6, 1),
            "all_extension_Mrays_s": round(int(counts[:16].sum()) / el / 1e6, 1),
            "ms_per_frame_synced": round(el_sync * 1e3, 3),
            "primary_rays": int(counts[0]), "bounce1_rays": int(counts[1]),
            "deep_rays": int(counts[2:16].sum()), "shadow_rays": int(counts[16]),
            "traceTime0_ms": round(st.traceTime0 * 1e3, 3), "traceTime1_ms": round(st.traceTime1 * 1e3, 3),
            "traceTimeX_ms": round(st.traceTimeX * 1e3, 3), "shadowTraceTime_ms": round(st.shadowTraceTime * 1e3, 3),
            "shadeTime_ms": round(st.shadeTime * 1e3, 3)}


def config3(args):
    t0 = time.perf_counter()
    sc = scene.room_scene(args.room_tris, args.width, args.height)
    core = RenderCore(device=0)
    core.setting("maxPathLength", 4)
    for kv in args.setting:
        core.setting(kv.split("=")[0], float(kv.split("=")[1]))
    sc.load_into(core)
    core.set_target(args.width, args.height, 1)
    setup = time.perf_counter() - t0
    r = measure(core, sc, args.frames, args.warmup)
    r.update({"config": "config3", "workload": f"room {sc.tri_count} tris, {args.width}x{args.height} 1 spp, maxPathLength 4",
              "setup_s": round(setup, 2), "scene": core.scene_info()})
    core.close()
    return r


def config5(args):
    t0 = time.perf_counter()
    sc = scene.instanced_scene(meshes=args.meshes, tris_per_mesh=args.mesh_tris, width=args.width, height=args.height)
    core = RenderCore(device=0)
    for kv in args.setting:
        core.setting(kv.split("=")[0], float(kv.split("=")[1]))
    sc.load_into(core)
    core.set_target(args.width, args.height, 8)
    setup = time.perf_counter() - t0

    def per_frame(i):
        scene.animate_instances(sc, i)
        for k, (mesh, T) in enumerate(sc.instances):
            core.set_instance(k, mesh, T)
        core.update_toplevel()

    r = measure(core, sc, args.frames, args.warmup, per_frame=per_frame)
    r.update({"config": "config5", "workload": f"{args.meshes} meshes x {args.mesh_tris} tris, per-frame instance "
                                               f"rotations + TLAS rebuild, {args.width}x{args.height} 8 spp",
              "setup_s": round(setup, 2), "scene": core.scene_info()})
    core.close()
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="3,5")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--room-tris", type=int, default=1_000_000)
    ap.add_argument("--meshes", type=int, default=100)
    ap.add_argument("--mesh-tris", type=int, default=100_000)
    ap.add_argument("--setting", action="append", default=[], help="name=value core setting")
    args = ap.parse_args()
    for c in args.configs.split(","):
        r = config3(args) if c.strip() == "3" else config5(args)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
