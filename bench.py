"""Benchmark: Mrays/s (primary + secondary) of the MI355X wavefront path tracer at 1080p 1 spp.

Workload (BASELINE.json configs[1]): 100k random triangles (xorshift32 seed
0x12345678, v0 ~ U[-5,5]^3, edge 0.5), camera (0,0,-12) -> +z, FOV 40, 16:9, material white 0.8
roughness 1.  One step = one complete frame of the wavefront path tracer through the reference
CoreAPI (camera rays, closest-hit BVH2 traversal, shade/extend/NEE, next bounce, shadow rays,
finalize) = primary + secondary extension rays (ENOUGH_BOUNCES = S_BOUNCED ends diffuse paths
after the second vertex, pathtracer.h:33,211), plus, for N > 1, the accumulator gather to rank 0.

Multi-GPU (weak scaling): with N ranks the frame is 1920 x (1080 N) pixels of the same 16:9 view,
dealt in 8-row bands round-robin, so each GPU traces a 1080p frame's worth of paths per step.

value = (primary + secondary rays of all ranks) x K / (max over ranks of the K-step time).
The roofline object is for the dominant kernel (closest-hit traversal) measured with HIP events
on the core's stream: algorithmic bytes per ray = 32 (ray) + 20 (hit) + 32 n_node + 36 n_tri with
n from the committed reference-traversal fixture (tests/golden/config2_visits.json).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402  (import before the core: one HIP runtime in the process)
import torch.distributed as dist  # noqa: E402

from lighthouse2_amd import scene  # noqa: E402
from lighthouse2_amd.core import RenderCore  # noqa: E402
from lighthouse2_amd.parallel import BAND, band_rows, gather_tiles  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print(msg, file=sys.stderr, flush=True)


def cpu_baseline(sc, width, height, seconds):
    """Reference CPU traversal (RenderCore_Bart, oracle/_ref) on a bounded sample of the same
    primary rays; falls back to the oracle's CPU traversal when the reference build is absent."""
    import ctypes as C
    threads = max(1, min(16, os.cpu_count() or 1))
    from oracle.oracle import Oracle
    orc = Oracle(threads=threads)
    sc.load_into(orc)
    orc.set_target(width, height, 1)
    orc.setting("epsilon", 1e-4)
    O4, D4, _ = orc.generate_eye_rays(sc.view, 0, 0)
    rng = np.random.default_rng(0)
    perm = rng.permutation(len(O4))
    ref = ROOT / "oracle" / "_ref" / "libbart_ref.so"
    if ref.exists():
        L = C.CDLL(str(ref))
        L.bart_build.restype = C.c_void_p
        L.bart_build.argtypes = [C.c_void_p, C.c_int]
        L.bart_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        tris = np.ascontiguousarray(sc.meshes[0], np.float32)
        h = L.bart_build(tris.ctypes.data, len(tris))
        kind = "reference"

        def trace(o, d):
            out = np.zeros((len(o), 4), np.float32)
            L.bart_trace(h, o.ctypes.data, d.ctypes.data, len(o), out.ctypes.data, None, threads)
    else:
        kind = "port"

        def trace(o, d):
            orc.trace_closest(np.concatenate([o, np.full((len(o), 1), 1e-4, np.float32)], 1),
                              np.concatenate([d, np.full((len(d), 1), 1e34, np.float32)], 1))
    done, t0, batch = 0, time.perf_counter(), 4096
    while time.perf_counter() - t0 < seconds:       # bounded sample: passes over the frame's rays, in random order
        start = done % len(perm)
        idx = perm[start:start + batch]
        trace(np.ascontiguousarray(O4[idx, :3]), np.ascontiguousarray(D4[idx, :3]))
        done += len(idx)
        batch = min(batch * 2, 262144)
    el = time.perf_counter() - t0
    return {"value": done / el / 1e6, "unit": "Mrays/s", "cores": threads, "kind": kind,
            "sample": f"{done} rays ({done / len(O4):.2f} passes over the {len(O4)} config-2 primary rays, 1080p), "
                      f"closest hit, {'RenderCore_Bart BVH2::Traverse' if kind == 'reference' else 'oracle trace_closest'}, "
                      f"{threads} threads, {el:.1f} s"}


def latest_pmc_traffic():
    """HBM bytes per closest-hit launch from the committed rocprofv3 --pmc summary (FETCH_SIZE doubled
    per the gfx950 calibration in MI355X_MICROARCH.md §HBM, WRITE_SIZE as is), if present."""
    files = sorted(glob.glob(str(ROOT / "profiles" / "*pmc_traffic*.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
        return d.get("bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--tris", type=int, default=100_000)
    ap.add_argument("--kernel-iters", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--setting", action="append", default=[], help="name=value core setting before loading (A/B runs)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    W, H = args.width, args.height * world
    sc = scene.config2_scene(n=args.tris, width=args.width, height=args.height)
    sc.view = scene.camera_view((0, 0, -12), (0, 0, 1), fov_deg=40, aspect=args.width / args.height, focal=5,
                                pixel_height=H)
    core = RenderCore(device=local)
    for kv in args.setting:
        k, v = kv.split("=")
        core.setting(k, float(v))
    t0 = time.perf_counter()
    sc.load_into(core)
    core.set_target(W, H, 1)
    core.set_tile_bands(rank, world, BAND)
    build_s = time.perf_counter() - t0
    rows = core.tile_rows()
    assert rows == len(band_rows(rank, world, H))
    tile = torch.empty((rows, W, 4), dtype=torch.float32, device=dev)

    def step():
        sc.render_frame(core, converge=1)     # Restart: the same paths every step
        core.pack_tile(tile.data_ptr())       # owned accumulator rows (waits for the frame)
        return gather_tiles(tile, rank, world, H)

    for _ in range(args.warmup):
        step()
    counts = core.ray_counts()
    st = core.stats()
    rays_rank = int(counts[0]) + int(counts[1])         # primary + secondary (CoreStats semantics)
    tot = torch.tensor([rays_rank, int(counts[2:16].sum()), int(counts[16])], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(tot)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    rays_total = int(tot[0].item())
    value = rays_total * args.steps / elapsed / 1e6

    if rank == 0:
        # ---- roofline of the dominant kernel: closest hit on the frame's bounce rays (per-ray traversal,
        # ~half the frame), and beside it the primary-ray launch (packet traversal when auto-selected) ----
        o4, d4, _ = core.generate_eye_rays(sc.view, 0, 0)
        perm = scene.tiled_order(W, H)        # the in-frame ray order (8x8 pixel block per wave)
        o4, d4 = np.ascontiguousarray(o4[perm]), np.ascontiguousarray(d4[perm])

        def launch(o, d, coherent):
            n = len(o)
            ro, rd = torch.from_numpy(o).to(dev), torch.from_numpy(d).to(dev)
            hits = torch.empty((n, 4), dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            core.setting("unitCoherent", 1 if coherent else 0)   # launched exactly as the frame launches it
            core.trace_closest_device(ro.data_ptr(), rd.data_ptr(), n, hits.data_ptr(), 2)
            ms = core.trace_closest_device(ro.data_ptr(), rd.data_ptr(), n, hits.data_ptr(), args.kernel_iters)
            core.setting("unitCoherent", 0)
            return ms, hits.cpu().numpy().view(np.uint32)

        def bytes_per_ray(name):
            fix = json.load(open(ROOT / "tests" / "golden" / name))
            return 32 + 20 + 32 * fix["mean_node_records"] + 36 * fix["mean_tri_tests"]

        ms_p, hits_p = launch(o4, d4, True)
        bo, bd = scene.bounce_rays(sc.meshes[0], o4, d4, hits_p)
        ms, _ = launch(bo, bd, False)
        n, n_p = len(bo), len(o4)
        bpr, bpr_p = bytes_per_ray("config2_bounce_visits.json"), bytes_per_ray("config2_visits.json")
        achieved = bpr * n / (ms * 1e-3) / 1e9
        achieved_p = bpr_p * n_p / (ms_p * 1e-3) / 1e9
        traffic = latest_pmc_traffic()
        info = core.scene_info()
        # RenderCore::UsePackets (auto): BVH + triangle footprint <= packetMaxMB (16 MiB)
        packets = (info["nodes"] * 64 + info["tris"] * 48) <= 16 * 1048576
        out = {
            "metric": "Mrays/s (primary+secondary) at 1080p 1spp",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"config2: {args.tris} random tris (xorshift32 0x12345678), {W}x{H} frame "
                                   f"({args.width}x{args.height} paths per GPU, {BAND}-row bands), 1 spp, "
                                   f"full wavefront frame (primary + bounce-1 rays)",
                       "frame": [W, H], "spp": 1, "tris": args.tris, "parallelism": f"tiles{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel": "k_trace_closest<false, 4> (per-ray BVH4 traversal, the core's default settings) on "
                                   "the frame's diffuse bounce rays, in-frame order", "kernel_ms": round(ms, 4),
                         "bytes_per_ray": round(bpr, 1), "rays_per_launch": n,
                         "bytes_model": "32 ray + 20 hit + 32 x node records + 36 x triangle tests of the reference "
                                        "traversal (tests/golden/config2_bounce_visits.json)"},
            "roofline_primary": {"bound": "hbm", "achieved": round(achieved_p, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(achieved_p / HBM_PEAK_GBS, 4),
                                 "kernel": ("k_trace_closest_packet (wave-uniform packet traversal)" if packets
                                            else "k_trace_closest<true, 4>") + " on the 1080p primary rays",
                                 "kernel_ms": round(ms_p, 4), "bytes_per_ray": round(bpr_p, 1), "rays_per_launch": n_p,
                                 "note": "per-ray byte model; a packet fetches each node once per 64 rays (scalar "
                                         "loads), so frac > 1 is possible and means the kernel is not HBM-bound"},
            "detail": {"primary_rays": int(counts[0]), "secondary_rays": int(counts[1]),
                       "deep_rays": int(counts[2:16].sum()), "shadow_rays": int(counts[16]),
                       "trace_Mrays_s_bounce": round(n / (ms * 1e-3) / 1e6, 1),
                       "trace_Mrays_s_primary": round(n_p / (ms_p * 1e-3) / 1e6, 1),
                       "trace_Mrays_s_frame": round(rays_total / world / ((st.traceTime0 + st.traceTime1) * 1e6), 1)
                       if st.traceTime0 + st.traceTime1 > 0 else None,
                       "traceTime0_ms": round(st.traceTime0 * 1e3, 4), "traceTime1_ms": round(st.traceTime1 * 1e3, 4),
                       "shadeTime_ms": round(st.shadeTime * 1e3, 4), "bvh_nodes": info["nodes"],
                       "bvh_depth": info["max_depth"], "setup_s": round(build_s, 3)},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(sc, args.width, args.height, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    core.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
