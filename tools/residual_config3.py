"""Where does the config-3 frame differ from the oracle?  

Renders the config-3 room (1M triangles, 1920x1080, 1 spp) on the GPU and with the CPU oracle at
maxPathLength 1..4 (and, at depth 4, with the path tail off), and prints per variant: relative L2 of the
accumulator, the number of pixels whose colour differs by more than 1e-3 relative, and the 20 worst pixels
with their values and their primary hit (triangle, material).  One JSON line per variant on stdout.
"""
from __future__ import annotations

import argparse
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402,F401  (one HIP runtime in the process)

from lighthouse2_amd import abi, scene  # noqa: E402
from lighthouse2_amd.core import RenderCore  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--depths", default="1,2,3,4")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--setting", action="append", default=[], help="name=value on the GPU core (after loading)")
    args = ap.parse_args()
    W, H = args.width, args.height
    sc = scene.room_scene(args.tris, W, H)
    tris = sc.meshes[0]
    core, o = RenderCore(device=0), Oracle()
    for t in (core, o):
        sc.load_into(t)
        t.set_target(W, H, 1)
    for kv in args.setting:
        k, v = kv.split("=")
        core.setting(k, float(v))
    # primary hits of every pixel (row-major eye rays of pass 0, the frame's R0 does not matter at pass 0 < 256)
    o.setting("epsilon", 1e-4)
    O4, D4, _ = o.generate_eye_rays(sc.view, 0, 0)
    prim = o.trace_closest(O4, D4)
    variants = [(int(d), ()) for d in args.depths.split(",")] + [(4, (("pathTail", 0),))]
    for depth, extra in variants:
        for t in (core, o):
            t.setting("maxPathLength", depth)
        core.setting("pathTail", 3)
        for k, v in extra:
            core.setting(k, v)
        sc.render_frame(core)
        sc.render_frame(o)
        cg, co = core.ray_counts(), o.ray_counts()
        ag, ao = core.accumulator()[..., :3], o.accumulator()[..., :3]
        d = np.abs(ag - ao).sum(-1)
        mag = np.abs(ao).sum(-1)
        rel = float(np.linalg.norm(ag - ao) / max(np.linalg.norm(ao), 1e-30))
        bad = d > 1e-3 * np.maximum(mag, 1e-3)
        worst = np.argsort(d.ravel())[::-1][:args.top]
        rows = []
        for p in worst:
            y, x = divmod(int(p), W)
            tri = int(prim[p, 1]) if prim[p, 1] != 0xFFFFFFFF else -1
            mat = int(tris[tri].view(np.uint32)[abi.TRI["material"]]) if tri >= 0 else -1
            rows.append({"x": x, "y": y, "gpu": [round(float(v), 6) for v in ag[y, x]], "oracle": [round(float(v), 6) for v in ao[y, x]],
                         "absdiff": round(float(d[y, x]), 6), "prim_tri": tri, "prim_mat": mat,
                         "prim_t": round(float(prim[p, 0].view(np.float32)), 5)})
        # share of the squared error in the worst pixels
        se = (d.ravel() ** 2)
        top_share = float(se[worst].sum() / max(se.sum(), 1e-30))
        print(json.dumps({"depth": depth, "extra": dict(extra), "counts_equal": bool(np.array_equal(cg, co)),
                          "rays": co[:5].tolist(), "shadow": int(co[16]), "rel_l2": rel, "bad_pixels": int(bad.sum()),
                          "top_sq_err_share": round(top_share, 4), "worst": rows}), flush=True)
    core.close()
    o.close()




def shadow_forensics(n_pixels: int = 10, tris_n: int = 1_000_000, W: int = 1920, H: int = 1080):
    """For the worst pixels of the depth-4 frame: the oracle's shadow rays of the pixel (orc_debug_pixel, one
    row rendered as a tile: the RNG uses global pixel indices) beside the GPU frame's queued shadow rays of the
    same pixel (lh2_core_debug_shadow_rays), and each ray's occlusion re-traced by the other implementation."""
    sc = scene.room_scene(tris_n, W, H)
    core, o = RenderCore(device=0), Oracle()
    for t in (core, o):
        sc.load_into(t)
        t.set_target(W, H, 1)
        t.setting("maxPathLength", 4)
    sc.render_frame(core)
    sc.render_frame(o)
    ag, ao = core.accumulator()[..., :3], o.accumulator()[..., :3]
    d = np.abs(ag - ao).sum(-1).ravel()
    worst = np.argsort(d)[::-1][:n_pixels]
    so, sd, sp = core.debug_shadow_rays(8_000_000)
    spx = sp[:, 3].view(np.uint32)
    for p in worst:
        y, x = divmod(int(p), W)
        o.set_tile(y, y + 1)
        o.debug_pixel(int(p))
        sc.render_frame(o)
        log = o.debug_log()
        o.set_tile(0, -1)
        o.debug_pixel(-1)
        orays = log[log[:, 0] == 1]
        verts = log[log[:, 0] == 0]
        g = np.nonzero(spx == p)[0]
        rec = {"x": x, "y": y, "absdiff": float(d[p]), "gpu_rgb": ag.reshape(-1, 3)[p].tolist(), "oracle_rgb": ao.reshape(-1, 3)[p].tolist(),
               "vertices": [{"L": int(v[1]), "t": float(v[2]), "tri": int(v[3:4].view(np.int32)[0]), "inst": int(v[4:5].view(np.int32)[0])} for v in verts],
               "oracle_shadow": [], "gpu_shadow": []}
        if len(orays):
            O4 = np.concatenate([orays[:, 3:6], np.zeros((len(orays), 1), np.float32)], 1)
            D4 = np.concatenate([orays[:, 6:9], orays[:, 9:10]], 1)
            occ_g = core.trace_any(O4, D4)
            for i, r in enumerate(orays):
                rec["oracle_shadow"].append({"L": int(r[1]), "occluded": int(r[2]), "gpu_retrace_occluded": int((occ_g[i >> 5] >> (i & 31)) & 1),
                                             "O": r[3:6].tolist(), "D": r[6:9].tolist(), "tmax": float(r[9]), "rgb": r[10:13].tolist()})
        if len(g):
            occ_o = o.trace_any(so[g], sd[g])
            for k, i in enumerate(g):
                rec["gpu_shadow"].append({"oracle_retrace_occluded": int((occ_o[k >> 5] >> (k & 31)) & 1), "O": so[i, :3].tolist(),
                                          "tmin": float(so[i, 3]), "D": sd[i, :3].tolist(), "tmax": float(sd[i, 3]), "rgb": sp[i, :3].tolist()})
        print(json.dumps(rec), flush=True)
    core.close()
    o.close()


if __name__ == "__main__":
    if "--forensics" in sys.argv:
        shadow_forensics()
    else:
        main()
