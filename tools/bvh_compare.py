"""CPU binned-SAH BLAS builder vs GPU PLOC builder (setting gpuBuild), per scene: build time
(SetGeometry of every mesh), node count / depth, and the frame time and trace times of the same
1080p frame traced over each tree.  One JSON line per (scene, builder)."""
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


def run(name, sc, builder, spp, frames, settings):
    core = RenderCore(device=0)
    core.setting("gpuBuild", builder)
    for k, v in settings.items():
        core.setting(k, v)
    t0 = time.perf_counter()
    sc.load_into(core)
    core.sync()
    build = time.perf_counter() - t0
    core.set_target(1920, 1080, spp)
    for i in range(2):
        sc.render_frame(core)
        core.sync()
    t0 = time.perf_counter()
    for i in range(frames):
        sc.render_frame(core)
        core.sync()
    ms = (time.perf_counter() - t0) / frames * 1e3
    st = core.stats()
    info = core.scene_info()
    out = {"scene": name, "builder": "gpu-ploc" if builder else "cpu-sah", "load_s": round(build, 3),
           "bvhBuildTime_s": round(st.bvhBuildTime, 3), "nodes": info["nodes"], "max_depth": info["max_depth"],
           "ms_per_frame": round(ms, 3), "traceTime0_ms": round(st.traceTime0 * 1e3, 3),
           "traceTime1_ms": round(st.traceTime1 * 1e3, 3), "shadowTraceTime_ms": round(st.shadowTraceTime * 1e3, 3)}
    core.close()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", default="config2,room,instanced")
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--builders", default="0,1")
    a = ap.parse_args()
    for name in a.scenes.split(","):
        if name == "config2":
            sc = scene.config2_scene(n=100_000, width=1920, height=1080)
            sc.view = scene.camera_view((0, 0, -12), (0, 0, 1), fov_deg=40, aspect=16 / 9, focal=5, pixel_height=1080)
            spp, st = 1, {}
        elif name == "room":
            sc = scene.room_scene(1_000_000, 1920, 1080)
            spp, st = 1, {"maxPathLength": 4}
        else:
            sc = scene.instanced_scene(meshes=20, tris_per_mesh=100_000, width=1920, height=1080, grid=5)
            spp, st = 2, {}
        for b in a.builders.split(","):
            run(name, sc, int(b), spp, a.frames, st)


if __name__ == "__main__":
    main()
