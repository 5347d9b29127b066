"""Generate the committed fixtures under tests/golden/ (run in the build container, never on the GPU box).

1. config2_visits.json - n_node / n_tri of the reference-style traversal (binned-SAH BVH2 per
   RenderCore_Bart/bvh.cpp:96-214, ordered and t-culled, as restated in oracle/pt_oracle.c) over the
   1920x1080 config-2 primary rays: the per-ray algorithmic byte model of SURVEY.md §8d / bench.py.
2. bart_config2_sample.npz - rays + closest-hit t / normal from the COMPILED reference traversal
   (oracle/_ref/libbart_ref.so built from /root/reference by oracle/Makefile.ref) on a 64x36
   subsample of config-2 primary rays: pins the oracle's traversal (tests/test_golden.py).
3. oracle_frames.npz - small oracle frames (accumulator + ray counts) used as regression goldens.
"""
from __future__ import annotations

import ctypes as C
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from lighthouse2_amd import scene  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

GOLD = ROOT / "tests" / "golden"


def visits_fixture():
    sc = scene.config2_scene(n=100_000, width=1920, height=1080)
    o = Oracle(threads=8)
    sc.load_into(o)
    o.set_target(1920, 1080, 1)
    o.setting("epsilon", 1e-4)
    O4, D4, _ = o.generate_eye_rays(sc.view, 0, 0)
    hits, vis = o.trace_closest(O4, D4, visits=True)
    d = {
        "scene": "config2 100k random tris, 1920x1080 primary rays, camera (0,0,-12)->+z FOV 40",
        "rays": int(len(O4)),
        "hit_fraction": float((hits[:, 1] != 0xFFFFFFFF).mean()),
        "mean_node_records": float(vis[:, 0].mean()),
        "mean_tri_tests": float(vis[:, 1].mean()),
        "node_record_bytes": 32, "tri_bytes": 36,
        "generator": "tools/make_fixtures.py (oracle restatement of RenderCore_Bart bvh.cpp:96-214, ordered t-culled traversal)",
    }
    (GOLD / "config2_visits.json").write_text(json.dumps(d, indent=1))
    print(d)
    # the frame's first bounce: diffuse rays from the primary hits (scene.bounce_rays, in-frame order)
    perm = scene.tiled_order(1920, 1080)
    O4, D4, hits = O4[perm], D4[perm], hits[perm]
    bo, bd = scene.bounce_rays(sc.meshes[0], O4, D4, hits)
    bhits, bvis = o.trace_closest(bo, bd, visits=True)
    b = {
        "scene": "config2 100k random tris; diffuse bounce rays (lighthouse2_amd.scene.bounce_rays, seed 1) "
                 "from the hits of the 1920x1080 primary rays",
        "rays": int(len(bo)),
        "hit_fraction": float((bhits[:, 1] != 0xFFFFFFFF).mean()),
        "mean_node_records": float(bvis[:, 0].mean()),
        "mean_tri_tests": float(bvis[:, 1].mean()),
        "node_record_bytes": 32, "tri_bytes": 36,
        "generator": d["generator"],
    }
    (GOLD / "config2_bounce_visits.json").write_text(json.dumps(b, indent=1))
    print(b)


def bart_fixture():
    ref = ROOT / "oracle" / "_ref" / "libbart_ref.so"
    if not ref.exists():
        print("reference build absent; skipping bart fixture")
        return
    L = C.CDLL(str(ref))
    L.bart_build.restype = C.c_void_p
    L.bart_build.argtypes = [C.c_void_p, C.c_int]
    L.bart_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
    sc = scene.config2_scene(n=100_000, width=1920, height=1080)
    tris = np.ascontiguousarray(sc.meshes[0], np.float32)
    h = L.bart_build(tris.ctypes.data, len(tris))
    o = Oracle(threads=8)
    sc.load_into(o)
    o.set_target(1920, 1080, 1)
    o.setting("epsilon", 1e-4)
    O4, D4, _ = o.generate_eye_rays(sc.view, 0, 0)
    sel = (np.arange(36)[:, None] * 30 * 1920 + np.arange(64)[None, :] * 30).ravel()
    org = np.ascontiguousarray(O4[sel, :3])
    dirs = np.ascontiguousarray(D4[sel, :3])
    out = np.zeros((len(sel), 4), np.float32)
    vis = np.zeros(len(sel), np.int32)
    L.bart_trace(h, org.ctypes.data, dirs.ctypes.data, len(sel), out.ctypes.data, vis.ctypes.data, 1)
    np.savez_compressed(GOLD / "bart_config2_sample.npz", org=org, dir=dirs, t=out[:, 0], normal=out[:, 1:4],
                        visits=vis, index=sel)
    print("bart sample: hit fraction", float((out[:, 0] < 1e30).mean()), "mean visits", float(vis.mean()))


def oracle_frames():
    frames = {}
    for name, sc in (("config2_light_96x54", scene.config2_scene(n=5000, width=96, height=54, sky=True, light=True)),
                     ("room_96x54", scene.room_scene(8000, 96, 54)),
                     ("textured_96x54", scene.textured_scene(96, 54, tess=8))):
        o = Oracle(threads=8)
        sc.load_into(o)
        o.set_target(96, 54, 1)
        sc.render_frame(o)
        frames[name + "_acc"] = o.accumulator()
        frames[name + "_counts"] = o.ray_counts()
    np.savez_compressed(GOLD / "oracle_frames.npz", **frames)
    print("oracle frames:", list(frames))


if __name__ == "__main__":
    GOLD.mkdir(parents=True, exist_ok=True)
    which = sys.argv[1:] or ["visits", "bart", "frames"]
    if "visits" in which:
        visits_fixture()
    if "bart" in which:
        bart_fixture()
    if "frames" in which:
        oracle_frames()
