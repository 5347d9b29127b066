"""BASELINE config 1: tinyapp + RenderCore_SoftRasterizer, default scene at
640 x 400, on the CPU - plumbing, frame time, no Mrays/s.

The scene is tinyapp's own (apps/tinyapp/main.cpp:34-45): the pica glTF diorama (76,274 triangles in 170
meshes, the root node rotated by RotateX(-pi/2)), the lego car OBJ (10,992 triangles, scale 10) and the
light quad (2 triangles, radiance 100, 100, 80, at y = 26, 6.9 x 6.9), read from the reference's assets
(apps/tinyapp/data) into tests/golden/config1_tinyapp.npz by tools/make_config1_fixture.py and converted
by scene.tinyapp_scene with the reference's mesh builders; the camera is tinyapp's default (no camera.xml
ships with the app).  The six glTF textures are applied as HostScene::AddScene converts them (one, missing from
the reference (.MISSING_LARGE_BLOBS), is a documented stand-in: scene.MISSING_TEXTURE_RGBA).

Measured, one JSON line:
  - the reference CPU rasterizer (RenderCore_SoftRasterizer/rasterizer.cpp, oracle/_ref/
    libsoftrast_ref.so built by oracle/Makefile.ref) rendering the scene: ms per frame, 1 thread
    (the reference is single-threaded), and the share of covered pixels (a non-empty image);
  - this core on cuda:0 rendering the same scene, same view, 1 spp path-traced frames with NEE
    (the reference core of config 1 rasterises; the comparison is of frame times, not images).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from lighthouse2_amd import abi, scene  # noqa: E402


def soft_rasterizer(sc: scene.Scene, width: int, height: int, seconds: float) -> dict:
    lib = ROOT / "oracle" / "_ref" / "libsoftrast_ref.so"
    if not lib.exists():
        return {"error": f"{lib} not built (oracle/Makefile.ref needs /root/reference)"}
    L = C.CDLL(str(lib))
    L.sr_create.restype = C.c_void_p
    L.sr_create.argtypes = [C.c_int, C.c_int]
    L.sr_set_geometry.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    L.sr_set_instance.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    L.sr_set_materials.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    L.sr_render.argtypes = [C.c_void_p, C.c_void_p]
    L.sr_pixels.restype = C.POINTER(C.c_uint32)
    L.sr_pixels.argtypes = [C.c_void_p]
    h = L.sr_create(width, height)
    keep = []
    for i, tris in enumerate(sc.meshes):
        T = len(tris)
        v = np.zeros((3 * T, 4), np.float32)
        for k, name in enumerate(("vertex0", "vertex1", "vertex2")):
            v[k::3, :3] = tris[:, abi.TRI[name]:abi.TRI[name] + 3]
        t = np.ascontiguousarray(tris)
        keep += [v, t]
        assert L.sr_set_geometry(h, i, v.ctypes.data, 3 * T, T, t.ctypes.data) == 0
    for i, (m, T) in enumerate(sc.instances):
        M = np.ascontiguousarray(T, np.float32)
        assert L.sr_set_instance(h, i, m, M.ctypes.data) == 0
    L.sr_set_textures.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    if sc.textures:
        keep += [np.ascontiguousarray(t.pixels) for t in sc.textures]
        descs = (abi.CoreTexDesc * len(sc.textures))(*[t.desc(k) for t, k in zip(sc.textures, keep[-len(sc.textures):])])
        assert L.sr_set_textures(h, C.cast(descs, C.c_void_p), len(sc.textures)) == 0
    mats = (abi.CoreMaterial * len(sc.materials))(*sc.materials)
    assert L.sr_set_materials(h, mats, len(sc.materials)) == 0
    view = sc.view
    L.sr_render(h, C.byref(view))
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        L.sr_render(h, C.byref(view))
        n += 1
    el = (time.perf_counter() - t0) / n
    px = np.ctypeslib.as_array(L.sr_pixels(h), shape=(width * height,))
    return {"ms_per_frame": round(el * 1e3, 3), "frames": n, "threads": 1,
            "covered_pixel_share": round(float((px != 0).mean()), 4)}


def mi355x_core(sc: scene.Scene, width: int, height: int, frames: int, settings=()) -> dict:
    import torch  # noqa: F401  (one HIP runtime in the process)
    from lighthouse2_amd.core import RenderCore
    t0 = time.perf_counter()
    core = RenderCore(device=0)
    for kv in settings:
        k, v = kv.split("=")
        core.setting(k, float(v))
    sc.load_into(core)
    core.set_target(width, height, 1)
    setup = time.perf_counter() - t0
    for _ in range(3):
        sc.render_frame(core, converge=1)
    core.sync()
    t0 = time.perf_counter()
    for _ in range(frames):
        sc.render_frame(core, converge=1)
    core.sync()
    el = (time.perf_counter() - t0) / frames
    counts = core.ray_counts()
    st = core.stats()
    acc = core.accumulator()
    core.close()
    return {"ms_per_frame": round(el * 1e3, 4), "frames": frames, "setup_s": round(setup, 3),
            "primary_rays": int(counts[0]), "bounce1_rays": int(counts[1]), "shadow_rays": int(counts[16]),
            "renderTime_ms": round(st.renderTime * 1e3, 4),
            "nonblack_pixel_share": round(float((acc[..., :3].sum(-1) > 0).mean()), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=400)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--frames", type=int, default=50)
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--setting", action="append", default=[], help="name=value core setting")
    args = ap.parse_args()
    sc = scene.tinyapp_scene(args.width, args.height)
    out = {"config": "config1", "workload": f"tinyapp default scene, {sc.tri_count} tris (pica glTF 76,274 in 170 "
           f"instances + legocar.obj 10,992 at scale 10 + 2-tri light quad; the six glTF textures), {args.width}x{args.height}",
           "soft_rasterizer_reference": soft_rasterizer(sc, args.width, args.height, args.cpu_seconds)}
    if not args.no_gpu:
        out["mi355x_core"] = mi355x_core(sc, args.width, args.height, args.frames, args.setting)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
