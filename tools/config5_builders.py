"""Config 5 (BASELINE configs[4]: 100 distinct 100k-triangle meshes, one instance each, per-frame rotations +
TLAS, 1080p 8 spp) per BLAS builder, on one MI355X: the core's scene setup time (SetGeometry x 100, the BLAS
builds, UpdateToplevel, SetTarget: what SynchronizeSceneData costs; the synthetic scene's generation in Python is
timed apart) and the frame time with that tree, as bench.py's config5 times it.  One JSON line per builder.

Builders (RenderCore settings, before SetGeometry): the default CPU binned SAH with spatial splits (SBVH, overlap
threshold bvhSpatial 1e-3, spatial splits tried in nodes of >= 64 references) and the DP BVH4 collapse; spatial splits
tried in every node (bvhSpatialMinRefs 0); the round-3 threshold 1e-5; no spatial splits (bvhSpatial 0); the
GPU PLOC builder (gpuBuild 1, bvh_gpu.hip), whose BVH2 the host collapses to BVH4 the same way.
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

BUILDERS = {"cpu_sbvh": (), "cpu_sbvh_min0": (("bvhSpatialMinRefs", 0.0),), "cpu_sbvh_min64": (("bvhSpatialMinRefs", 64.0),), "cpu_sbvh_1e-5": (("bvhSpatial", 1e-5),), "cpu_sah": (("bvhSpatial", 0.0),),
            "gpu_ploc": (("gpuBuild", 1.0),)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--builders", default="cpu_sbvh,cpu_sbvh_1e-5,cpu_sah,gpu_ploc")
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--meshes", type=int, default=100)
    args = ap.parse_args()
    t0 = time.perf_counter()
    sc = scene.instanced_scene(meshes=args.meshes, tris_per_mesh=100_000, width=1920, height=1080)
    gen = time.perf_counter() - t0
    for name in args.builders.split(","):
        core = RenderCore(device=0)
        for k, v in BUILDERS[name]:
            core.setting(k, v)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sc.load_into(core)
        core.set_target(1920, 1080, 8)
        core.sync()
        setup = time.perf_counter() - t0
        info = core.scene_info()

        def frame(i):
            scene.animate_instances(sc, i)
            for k, (mesh, T) in enumerate(sc.instances):
                core.set_instance(k, mesh, T)
            core.update_toplevel()
            sc.render_frame(core, converge=1 if i == 0 else 0)

        for i in range(args.warmup):
            frame(i)
        core.sync()
        t0 = time.perf_counter()
        for i in range(args.frames):
            frame(args.warmup + i)
        core.sync()
        ms = (time.perf_counter() - t0) / args.frames * 1e3
        st = core.stats()
        counts = core.ray_counts()
        print(json.dumps({"builder": name, "settings": dict(BUILDERS[name]), "scene_gen_s": round(gen, 2),
                          "setup_s": round(setup, 3), "bvh_nodes": info["nodes"], "bvh_depth": info["max_depth"],
                          "leaf_tris": info["tris"], "ms_per_frame": round(ms, 3),
                          "Mrays_s": round((int(counts[0]) + int(counts[1])) / ms / 1e3, 1),
                          "trace_ms": {"t0": round(st.traceTime0 * 1e3, 3), "t1": round(st.traceTime1 * 1e3, 3)}}),
              flush=True)
        core.close()


if __name__ == "__main__":
    main()
