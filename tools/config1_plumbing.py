"""BASELINE config 1: tinyapp + RenderCore_SoftRasterizer, default scene at
640 x 400, on the CPU - plumbing, frame time, no Mrays/s.

tinyapp's PrepareScene (apps/tinyapp/main.cpp:34-45) loads the pica glTF (76,274 triangles), the
legocar OBJ (10,992 faces, scale 10) and a light quad (2 triangles, radiance 100, 100, 80).  The
assets are missing from the reference (.MISSING_LARGE_BLOBS), so the scene here is synthetic with
the same triangle counts: a 76,274-triangle cloud (the config-2 generator), a 10,992-triangle cloud
of 1/10 the size instanced at scale 10, and the light quad.

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


def tinyapp_scene(width: int = 640, height: int = 400) -> scene.Scene:
    body = scene.random_triangles(76_274, seed=0x2468ACE1, edge=0.5, spread=10.0)
    car = scene.random_triangles(10_992, seed=0x13579BDF, edge=0.05, spread=1.0)
    car.view(np.uint32)[:, abi.TRI["material"]] = 1
    mats = [abi.make_material((0.8, 0.8, 0.8), roughness=1.0), abi.make_material((0.8, 0.2, 0.1), roughness=1.0),
            abi.make_material((100.0, 100.0, 80.0))]
    quad = scene.quad_tris((0, -1, 0), (0, 9.0, 0), 4, 4, 2)
    quad.view(np.int32)[:, abi.TRI["ltriIdx"]] = [0, 1]
    S = np.diag([10.0, 10.0, 10.0, 1.0]).astype(np.float32)
    S[:3, 3] = (0.0, -2.0, 0.0)
    sc = scene.Scene(meshes=[body, car, quad],
                     instances=[(0, np.eye(4, dtype=np.float32)), (1, S), (2, np.eye(4, dtype=np.float32))],
                     materials=mats, name="tinyapp-like")
    sc.area_lights = [scene.light_from_tri(quad[i], i, 2, (100.0, 100.0, 80.0)) for i in range(2)]
    sc.view = scene.camera_view((0, 0, -14), (0, 0, 1), fov_deg=40, aspect=width / height, focal=5,
                                pixel_height=height)
    return sc


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


def mi355x_core(sc: scene.Scene, width: int, height: int, frames: int) -> dict:
    import torch  # noqa: F401  (one HIP runtime in the process)
    from lighthouse2_amd.core import RenderCore
    t0 = time.perf_counter()
    core = RenderCore(device=0)
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
    args = ap.parse_args()
    sc = tinyapp_scene(args.width, args.height)
    out = {"config": "config1", "workload": f"tinyapp-like scene, {sc.tri_count} tris "
           f"(76,274 + 10,992 at scale 10 + 2-tri light quad; synthetic: the assets are missing), {args.width}x{args.height}",
           "soft_rasterizer_reference": soft_rasterizer(sc, args.width, args.height, args.cpu_seconds)}
    if not args.no_gpu:
        out["mi355x_core"] = mi355x_core(sc, args.width, args.height, args.frames)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
