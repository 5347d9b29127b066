"""Microbenchmark of the closest-hit traversal kernel (k_trace_closest) on the config-2 scene.

Ray sets: the 1080p primary rays, and diffuse 'bounce' rays (cosine-weighted around the face normal
of each primary hit, origin offset by 1e-4 along the normal), i.e. what the first shade pass emits.
Used for kernel tuning and as the target process of the rocprofv3 --pmc passes.
"""
from __future__ import annotations

import argparse
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from lighthouse2_amd import abi, scene  # noqa: E402
from lighthouse2_amd.core import RenderCore  # noqa: E402


bounce_rays = scene.bounce_rays   # shared with bench.py and tools/make_fixtures.py


def scene_tris_box(sc):
    """The box of every triangle vertex of the scene's first mesh (config 2: the whole scene)."""
    t = np.asarray(sc.meshes[0])
    v = np.concatenate([t[:, 32:35], t[:, 36:39], t[:, 40:43]], 0)
    return v.min(0), v.max(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tris", type=int, default=100_000)
    ap.add_argument("--set", default="both")
    ap.add_argument("--scene", default="config2", choices=["config2", "room"])
    # defaults = the core's (RenderCore refillOther / leafBatch: primary rays traced per ray take the same)
    ap.add_argument("--refill", type=int, default=None, help="default: the core's setting")
    ap.add_argument("--leaf-batch", type=int, default=None)
    ap.add_argument("--no-frame-launch", action="store_true",
                    help="do not set unitCoherent=1 for the primary set (the frame's launch: packets when auto-selected)")
    ap.add_argument("--pre-setting", action="append", default=[], help="name=value set before loading (BVH build)")
    ap.add_argument("--setting", action="append", default=[], help="name=value core setting")
    ap.add_argument("--sweep", action="store_true", help="refill x leafBatch grid")
    ap.add_argument("--no-chord-order", action="store_true", help="bounce rays in plain in-frame order")
    ap.add_argument("--tile-cost", default=None, help="int32 per-tile cost file: also time the packets in LPT order")
    ap.add_argument("--tile-chord", type=float, action="append", default=[],
                    help="also time the primary packets reordered by their centre ray's chord (fraction F last)")
    ap.add_argument("--chord", type=float, action="append", default=[],
                    help="also time the bounce rays with the shortest-chord fraction F of each segment moved to its end")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    # --scene room: config 3's room (1M triangles, a closed room of tessellated walls and clutter) instead of config 2's soup
    sc = scene.room_scene(args.tris, 1920, 1080) if args.scene == "room" else scene.config2_scene(n=args.tris)
    core = RenderCore(device=0)
    for s in args.pre_setting:               # build parameters: before the scene is loaded
        k, v = s.split("=")
        core.setting(k, float(v))
    sc.load_into(core)
    core.set_target(1920, 1080, 1)
    core.setting("epsilon", 1e-4)
    for s in args.setting:
        k, v = s.split("=")
        core.setting(k, float(v))
    O4, D4, _ = core.generate_eye_rays(sc.view, 0, 0)
    perm = scene.tiled_order(1920, 1080)    # in-frame order of the primary rays (k_camera, tiledRays)
    sets = {"primary": (np.ascontiguousarray(O4[perm]), np.ascontiguousarray(D4[perm]))}
    if args.tile_cost:
        # primary packets per segment in descending order of a per-tile cost file (int32 per 8x8 tile,
        # tile order = slot order; tools/bvh_quality.cpp TILES_OUT): longest-processing-time first
        cost = np.fromfile(args.tile_cost, dtype=np.int32)
        po, pd = sets["primary"]
        ntile = len(po) // 64
        assert len(cost) == ntile
        seg = (ntile + 7) // 8
        tiles = np.concatenate([np.arange(c * seg, min(ntile, (c + 1) * seg))[np.argsort(-cost[c * seg:min(ntile, (c + 1) * seg)], kind="stable")]
                                for c in range(8)])
        rays = (tiles[:, None] * 64 + np.arange(64)[None, :]).reshape(-1)
        sets["primary_cost"] = (np.ascontiguousarray(po[rays]), np.ascontiguousarray(pd[rays]))
    for f in args.tile_chord:
        # the primary packets (64-ray tiles) reordered per segment by the chord of their centre ray through
        # the scene box: the shortest fraction f last (f >= 1: every segment sorted by descending chord)
        po, pd = sets["primary"]
        lo_, hi_ = scene_tris_box(sc)
        ctr = np.arange(32, len(po), 64)
        with np.errstate(divide="ignore", invalid="ignore"):
            t1 = np.minimum.reduce([np.maximum((lo_[k] - po[ctr, k]) / pd[ctr, k], (hi_[k] - po[ctr, k]) / pd[ctr, k]) for k in range(3)])
        ntile = len(ctr)
        seg = (ntile + 7) // 8
        order = []
        for c in range(8):
            ti = np.arange(c * seg, min(ntile, (c + 1) * seg))
            if f >= 1.0:
                order.append(ti[np.argsort(-t1[ti], kind="stable")])
            else:
                cut = np.quantile(t1[ti], f)
                order += [ti[t1[ti] > cut], ti[t1[ti] <= cut]]
        tiles = np.concatenate(order)
        rays = (tiles[:, None] * 64 + np.arange(64)[None, :]).reshape(-1)
        sets[f"primary_chord{f}"] = (np.ascontiguousarray(po[rays]), np.ascontiguousarray(pd[rays]))
    if args.set in ("both", "bounce", "bounce_sorted"):
        hits = core.trace_closest(O4, D4)
        bo, bd = bounce_rays(sc.meshes[0], O4[perm], D4[perm], hits[perm])   # compacted, in-frame order
        plain = (bo, bd)
        # as the frame's trace takes them: two-ended segments (chordSplit; --no-chord-order: plain in-frame)
        if not args.no_chord_order:
            order = scene.chord_order(bo, bd, *scene.mesh_box(sc.meshes[0]), core.get_setting("chordSplit"))
            bo, bd = np.ascontiguousarray(bo[order]), np.ascontiguousarray(bd[order])
        sets["bounce"] = (bo, bd)
        for f in args.chord:
            # the chord of each ray through the scene box; per segment (the launch's eighths), the
            # shortest-chord fraction f goes last, both parts in their in-frame order
            bo, bd = plain
            v = scene_tris_box(sc)
            with np.errstate(divide="ignore", invalid="ignore"):
                t1 = np.minimum.reduce([np.maximum((v[0][k] - bo[:, k]) / bd[:, k], (v[1][k] - bo[:, k]) / bd[:, k]) for k in range(3)])
            n = len(bo)
            seg = (n + 7) // 8
            order = []
            for c in range(8):
                idx = np.arange(c * seg, min(n, (c + 1) * seg))
                if len(idx) == 0:
                    continue
                cut = np.quantile(t1[idx], f)
                order.append(idx[t1[idx] > cut])
                order.append(idx[t1[idx] <= cut])
            if f >= 1.0:
                # f >= 1: every segment fully sorted by descending chord
                order = [np.arange(c * seg, min(n, (c + 1) * seg))[np.argsort(-t1[c * seg:min(n, (c + 1) * seg)], kind="stable")] for c in range(8)]
            order = np.concatenate(order)
            sets[f"bounce_chord{f}"] = (np.ascontiguousarray(bo[order]), np.ascontiguousarray(bd[order]))
        if args.set in ("both", "bounce_sorted"):
            # sorted by (direction octant, Morton code of the origin): coherent groups of 64 rays
            bo, bd = sets["bounce"]
            lo, hi = bo[:, :3].min(0), bo[:, :3].max(0)
            q = np.clip(((bo[:, :3] - lo) / np.maximum(hi - lo, 1e-9) * 1023).astype(np.int64), 0, 1023)
            def spread(x):
                x = (x | (x << 16)) & 0x030000FF; x = (x | (x << 8)) & 0x0300F00F
                x = (x | (x << 4)) & 0x030C30C3; return (x | (x << 2)) & 0x09249249
            m = (spread(q[:, 0]) << 2) | (spread(q[:, 1]) << 1) | spread(q[:, 2])
            octant = ((bd[:, 0] < 0).astype(np.int64) << 2) | ((bd[:, 1] < 0).astype(np.int64) << 1) | (bd[:, 2] < 0)
            order = np.argsort((octant << 30) | m, kind="stable")
            sets["bounce_sorted"] = (np.ascontiguousarray(bo[order]), np.ascontiguousarray(bd[order]))
            # direction octant only (stable: in-frame order within an octant): globally, and per segment
            order = np.argsort(octant, kind="stable")
            sets["bounce_oct"] = (np.ascontiguousarray(bo[order]), np.ascontiguousarray(bd[order]))
            n = len(bo)
            seg = (n + 7) // 8
            order = np.concatenate([c * seg + np.argsort(octant[c * seg:min(n, (c + 1) * seg)], kind="stable") for c in range(8)])
            sets["bounce_octseg"] = (np.ascontiguousarray(bo[order]), np.ascontiguousarray(bd[order]))
            if args.set == "bounce_sorted":
                del sets["bounce"]
    if args.sweep:
        # refill x leafBatch grid per ray set, one process (scene loaded once)
        for name, (o, d) in sets.items():
            n = len(o)
            ro, rd = torch.from_numpy(o).to(dev), torch.from_numpy(d).to(dev)
            h = torch.empty((n, 4), dtype=torch.int32, device=dev)
            for rf in (4, 8, 16, 32, 48, 64):
                for lb in (0, 4, 8, 16, 32):
                    core.setting("refill", rf)
                    core.setting("leafBatch", lb)
                    core.trace_closest_device(ro.data_ptr(), rd.data_ptr(), n, h.data_ptr(), 1)
                    ms = core.trace_closest_device(ro.data_ptr(), rd.data_ptr(), n, h.data_ptr(), args.iters)
                    print(json.dumps({"set": name, "refill": rf, "leafBatch": lb, "ms": round(ms, 4)}), flush=True)
        core.close()
        return
    res = {}
    for name, (o, d) in sets.items():
        if args.set not in ("both", name) and not (args.set == "bounce_sorted" and name == "bounce_sorted") \
                and not name.startswith("bounce_chord") and not name.startswith("primary_"):
            continue
        n = len(o)
        prim = name.startswith("primary")
        if args.refill is not None:
            core.setting("refill", args.refill)
        if args.leaf_batch is not None:
            core.setting("leafBatch", args.leaf_batch)
        if not args.no_frame_launch:
            core.setting("unitCoherent", 1 if prim else 0)
        ro, rd = torch.from_numpy(o).to(dev), torch.from_numpy(d).to(dev)
        h = torch.empty((n, 4), dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        core.trace_closest_device(ro.data_ptr(), rd.data_ptr(), n, h.data_ptr(), 2)
        ms = core.trace_closest_device(ro.data_ptr(), rd.data_ptr(), n, h.data_ptr(), args.iters)
        res[name] = {"rays": n, "ms": round(ms, 4), "Mrays_s": round(n / ms / 1e3, 1)}
    res["scene"] = core.scene_info()
    print(json.dumps(res))
    core.close()


if __name__ == "__main__":
    main()
