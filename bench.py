"""Benchmark: Mrays/s (primary + secondary) of the MI355X wavefront path tracer at 1080p 1 spp.

Workload (BASELINE.json configs[1]): 100k random triangles (xorshift32 seed
0x12345678, v0 ~ U[-5,5]^3, edge 0.5), camera (0,0,-12) -> +z, FOV 40, 16:9, material white 0.8
roughness 1.  One step = one complete frame of the wavefront path tracer through the reference
CoreAPI (camera rays, closest-hit BVH traversal, shade/extend/NEE, next bounce, shadow rays,
finalize) = primary + secondary extension rays (ENOUGH_BOUNCES = S_BOUNCED ends diffuse paths
after the second vertex, pathtracer.h:33,211), plus, for N > 1, the pack of the owned rows and their
gather to rank 0 (one rank keeps the finished frame in the core's frame buffer).

Multi-GPU, two measurements per run:
  value (weak scaling): with N ranks the frame is 1920 x (1080 N) pixels of the same 16:9 view,
    dealt in 8-row bands round-robin, so each GPU traces a 1080p frame's worth of paths per step;
  "config4" (strong scaling, BASELINE.json configs[3]): the config-3 scene (1M-triangle room,
    maxPathLength 4, lights) at 3840 x 2160, 1 spp, the same frame split across the N ranks in
    8-row bands, gathered to rank 0 over RCCL every frame.
Both: time = max over ranks of the K-step time between barriers; value = rays of all ranks / time.

roofline: the dominant kernel (the per-ray BVH4 closest-hit traversal of the frame's bounce rays),
timed live with the HIP events its launches record, priced by the resource the counters say binds
it: VALU issue (SQ_INSTS_VALU per launch, rocprofv3 --pmc, profiles/*_pmc_trace_sq.json) against
the chip's VALU issue peak.  The HBM view is kept beside it: measured bytes per launch (FETCH_SIZE /
WRITE_SIZE passes, profiles/*_pmc_traffic.json) and the SURVEY §8(d) algorithmic byte model.
"""
from __future__ import annotations

import argparse
import glob
import json
import re
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402  (import before the core: one HIP runtime in the process)
import torch.distributed as dist  # noqa: E402

from lighthouse2_amd import build_info, scene  # noqa: E402
from lighthouse2_amd.core import RenderCore  # noqa: E402
from lighthouse2_amd.parallel import BAND, TileGather  # noqa: E402

LH2_CONVERGE, LH2_RESTART = 0, 1   # include/lh2_core_types.h (Convergence, core_api_base.h)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
SIMDS, CLOCK_GHZ = 256 * 4, 2.4
# the per-ray closest-hit kernel of incoherent rays per traversal loop version (rocprofv3 names)
TRACE_KERNEL = {1: "k_trace_closest<", 7: "k_trace_closest4d"}


def log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print(msg, file=sys.stderr, flush=True)


def newest(pattern, pred=lambda d: True):
    """(path, dict) of the newest committed profile summary matching pattern and pred (tags r<round><letters>_: by
    round, then by the letters as a base-26 count, so r04ah follows r04z)."""
    def tag(f):
        m = re.match(r"r(\d+)([a-z]*)_", pathlib.Path(f).name)
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    for f in sorted(glob.glob(str(ROOT / "profiles" / pattern)), key=tag, reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if pred(d):
            return pathlib.Path(f).name, d
    return None, None


def valu_cycles_per_instruction():
    """SIMD cycles per wave64 VALU instruction at 8 waves per SIMD, measured per instruction class by tools/valu_rate
    (round 6: per-SIMD s_memtime spans, 16 independent chains per lane, the timed loops' ISA committed beside the numbers,
    profiles/*_valu_rate.jsonl + *_valu_rate_isa.txt).  Returns (fastest class: the VOP2 adds / multiplies, the guide's
    "2 cycles on a SIMD-32", which is the roofline peak; the node step's own instruction mix; the file).  VOP3 forms
    (fma, max3, pk_fma, cndmask_e64, compares into SGPRs), byte conversions and ldexp take ~4 cycles, v_rcp 8, so a kernel
    issuing only VOP3 work tops out near half the peak; the mix ceiling is reported beside it.  Without a probe file:
    the guide's 2 cycles for both."""
    def tag(f):
        m = re.match(r"r(\d+)([a-z]*)_", pathlib.Path(f).name)
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    files = sorted(glob.glob(str(ROOT / "profiles" / "*_valu_rate.jsonl")), key=tag)
    for f in reversed(files):
        rows = [json.loads(line) for line in open(f) if line.strip().startswith("{")]
        rows = [r for r in rows if r.get("waves_per_simd") == 8 and r.get("cycles_per_wave_inst")]
        mix = [r["cycles_per_wave_inst"] for r in rows if r["mode"] == "mix"]
        if rows and mix:
            return min(r["cycles_per_wave_inst"] for r in rows), mix[0], pathlib.Path(f).name
    return 2.0, 2.0, None


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


def apply_settings(core, args):
    """--setting name=value (A/B runs): applied to every core the bench creates, before its scene is loaded."""
    for kv in args.setting:
        k, v = kv.split("=")
        core.setting(k, float(v))
    return core


def timed_frames(core, sc, gather, steps, warmup, world, dev, per_frame=None):
    """warmup + steps frames (render; N > 1: pack the owned rows, gather); returns (max-over-ranks
    seconds, rays of all ranks per frame [primary + bounce 1, deeper, shadow], this rank's counts).
    With one rank the finished frame is the core's own frame buffer: there is nothing to exchange."""
    first = [True]

    def step():
        # a still camera converging, as imguiapp renders a still scene (apps/imguiapp/main.cpp:188-204: Restart only
        # when the camera moved, a material changed or an animation ran): the first frame restarts, every later one
        # accumulates a new sample with new random numbers, so no frame repeats the previous one's paths (the
        # heavy-first packet order is last frame's costs).  tinyapp's animated loop (a Restart every frame) is
        # timed beside it: "config2_restart
        sc.render_frame(core, converge=LH2_RESTART if first[0] else LH2_CONVERGE)
        first[0] = False
        if world == 1:
            return None
        core.pack_tile(gather.send.data_ptr())    # owned accumulator rows (ordered with torch's stream)
        return gather.gather()

    for _ in range(warmup):
        step()
    counts = core.ray_counts()
    tot = torch.tensor([int(counts[0]) + int(counts[1]), int(counts[2:16].sum()), int(counts[16])], dtype=torch.int64,
                       device=dev)
    if world > 1:
        dist.all_reduce(tot)
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return float(el.item()), [int(x) for x in tot.tolist()], counts


def config4(args, rank, world, local, dev):
    """BASELINE configs[3]: 4K 1 spp of the config-3 room, the frame split across the ranks (strong
    scaling), RCCL gather of the accumulator rows to rank 0 every frame."""
    W4, H4 = 3840, 2160
    sc = scene.room_scene(args.room_tris, W4, H4)
    core = RenderCore(device=local)
    core.setting("maxPathLength", 4)
    for kv in args.setting:
        k, v = kv.split("=")
        core.setting(k, float(v))
    sc.load_into(core)
    core.set_target(W4, H4, 1)
    core.set_tile_bands(rank, world, BAND)
    g = TileGather(rank, world, W4, H4, dev)
    assert core.tile_rows() == g.rows
    el, tot, _ = timed_frames(core, sc, g, args.config4_steps, args.warmup, world, dev)
    core.close()
    return {"workload": f"config4: room {sc.tri_count} tris (config-3 scene, maxPathLength 4, 2 area lights), "
                        f"{W4}x{H4} 1 spp, frame split across {world} GPU(s) in {BAND}-row bands, RCCL gather of the "
                        f"accumulator rows to rank 0 per frame",
            "scaling": "strong", "n_gpus": world, "steps": args.config4_steps,
            "value": round(tot[0] * args.config4_steps / el / 1e6, 3), "unit": "Mrays/s (primary+secondary)",
            "ms_per_frame": round(el / args.config4_steps * 1e3, 4),
            "rays_per_frame": {"primary_plus_bounce1": tot[0], "deeper": tot[1], "shadow": tot[2]}}


def single_gpu_frames(core, sc, steps, warmup, per_frame=None):
    """frames timed like the step loop (K frames between two synchronisations, the host queueing frame
    i + 1 while the GPU renders frame i); a converging still camera (frame 0 restarts), per_frame(i) first (config 5's instance
    updates).  Returns (seconds per frame, ray counts of the last frame)."""
    def frame(i):
        if per_frame:
            per_frame(i)
        sc.render_frame(core, converge=LH2_RESTART if i == 0 else LH2_CONVERGE)   # as timed_frames
    for i in range(warmup):
        frame(i)
    core.sync()
    counts = core.ray_counts()
    t0 = time.perf_counter()
    for i in range(steps):
        frame(warmup + i)
    core.sync()
    return (time.perf_counter() - t0) / steps, counts


def config2_restart(args, local):
    """The config-2 frame as tinyapp's animated main loop renders it (apps/tinyapp/main.cpp:98-118): every frame a
    SetNodeTransform of one node (here the scene's one instance: a small rotation, SetInstance + UpdateToplevel,
    rendersystem.cpp:143-174) and Render(Restart) (camMoved is set every frame).  The instance-only UpdateToplevel writes
    the TLAS slot no frame in flight reads and the restart zeroes the accumulator on the core stream, so these frames
    overlap like converging ones (DESIGN §4 "Animated frames")."""
    t0 = time.perf_counter()
    sc = scene.config2_scene(n=args.tris, width=args.width, height=args.height)
    core = RenderCore(device=local)
    for kv in args.setting:
        k, v = kv.split("=")
        core.setting(k, float(v))
    sc.load_into(core)
    core.set_target(args.width, args.height, 1)
    setup = time.perf_counter() - t0
    mesh0 = sc.instances[0][0]

    def frame(i):
        core.set_instance(0, mesh0, scene.rotation_y(1e-3 * i))   # tinyapp: r += deltaTime * 0.3 per frame
        core.set_instance(1, -1, None)                             # UpdateSceneGraph's end of the instance list
        core.update_toplevel()
        sc.render_frame(core, converge=LH2_RESTART)

    for i in range(args.warmup):
        frame(i)
    core.sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        frame(args.warmup + i)
    core.sync()
    el = (time.perf_counter() - t0) / args.steps
    counts = core.ray_counts()
    r = frame_record(f"config2_restart: {args.tris} random tris, {args.width}x{args.height} 1 spp, Restart + "
                     f"SetInstance + UpdateToplevel every frame (tinyapp's animated loop)", el, counts, core.stats(), setup)
    core.close()
    return r


def frame_record(workload, el, counts, st, setup_s):
    return {"workload": workload, "ms_per_frame": round(el * 1e3, 4),
            "value": round((int(counts[0]) + int(counts[1])) / el / 1e6, 3), "unit": "Mrays/s (primary+secondary)",
            "all_extension_Mrays_s": round(int(counts[:16].sum()) / el / 1e6, 1),
            "rays_per_frame": {"primary": int(counts[0]), "bounce1": int(counts[1]), "deeper": int(counts[2:16].sum()),
                               "shadow": int(counts[16])},
            "coreStats_ms": {"trace0": round(st.traceTime0 * 1e3, 4), "trace1": round(st.traceTime1 * 1e3, 4),
                             "traceX": round(st.traceTimeX * 1e3, 4), "shadow": round(st.shadowTraceTime * 1e3, 4),
                             "shade": round(st.shadeTime * 1e3, 4)},
            "setup_s": round(setup_s, 2)}


def config3(args, local):
    """BASELINE configs[2]: full wavefront path trace, maxPathLength 4, the 1M-triangle procedural room
    (specular chains, glass, two area lights: NEE + shadow rays), 1080p 1 spp, one GPU."""
    t0 = time.perf_counter()
    sc = scene.room_scene(args.room_tris, 1920, 1080)
    core = apply_settings(RenderCore(device=local), args)
    core.setting("maxPathLength", 4)
    sc.load_into(core)
    core.set_target(1920, 1080, 1)
    setup = time.perf_counter() - t0
    el, counts = single_gpu_frames(core, sc, args.config_steps, args.warmup)
    r = frame_record(f"config3: room {sc.tri_count} tris, 1920x1080 1 spp, maxPathLength 4, 2 area lights",
                     el, counts, core.stats(), setup)
    core.close()
    return r


def config5(args, local):
    """BASELINE configs[4]: 100 distinct 100k-triangle meshes (10M triangles), one instance each, new
    seeded rotations of every instance each frame (SetInstance x 100 + UpdateToplevel inside the timed
    frame), 1080p 8 spp (16,588,800 paths), one GPU."""
    t0 = time.perf_counter()
    sc = scene.instanced_scene(meshes=100, tris_per_mesh=100_000, width=1920, height=1080)
    gen = time.perf_counter() - t0
    core = apply_settings(RenderCore(device=local), args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()      # the core's setup (SynchronizeSceneData: SetGeometry x 100, BLAS builds, TLAS)
    sc.load_into(core)
    core.set_target(1920, 1080, 8)
    core.sync()
    setup = time.perf_counter() - t0

    def per_frame(i):
        scene.animate_instances(sc, i)
        for k, (mesh, T) in enumerate(sc.instances):
            core.set_instance(k, mesh, T)
        core.update_toplevel()

    el, counts = single_gpu_frames(core, sc, args.config_steps, args.warmup, per_frame)
    r = frame_record("config5: 100 meshes x 100k tris, per-frame instance rotations + TLAS rebuild, 1920x1080 8 spp",
                     el, counts, core.stats(), setup)
    r["scene_gen_s"] = round(gen, 2)   # the synthetic scene's generation in Python (not the core's)
    core.close()
    return r


def config4_incore(args, ndev):
    """Config 4 through the path an unchanged application uses: ONE process, one core (CreateCore /
    RenderSystem, core_api_base.cpp:97-132) with setting "deviceCount" = the GPUs of the run, which
    partitions the 4K frame over the devices itself and gathers the accumulator rows to device 0 by
    xGMI peer copies (csrc/multidevice.cpp).  Each frame is driven as RenderSystem::Render drives it:
    six Setting calls, then Render (rendersystem.cpp:228-238).  At one GPU it is the plain core."""
    W4, H4 = 3840, 2160
    t0 = time.perf_counter()
    sc = scene.room_scene(args.room_tris, W4, H4)
    core = apply_settings(RenderCore(device=0), args)
    if ndev > 1:
        core.setting("deviceCount", ndev)
    core.setting("maxPathLength", 4)
    sc.load_into(core)
    core.set_target(W4, H4, 1)
    setup = time.perf_counter() - t0

    def frame(i):
        for name, v in (("epsilon", 1e-4), ("clampValue", 10.0), ("clampDirect", 1.0), ("clampIndirect", 1.0),
                        ("filter", 0.0), ("TAA", 0.0)):
            core.setting(name, v)
        core.render(sc.view, LH2_RESTART if i == 0 else LH2_CONVERGE)   # as timed_frames

    for i in range(args.warmup):
        frame(i)
    core.sync()
    counts = core.ray_counts()
    t0 = time.perf_counter()
    for i in range(args.config4_steps):
        frame(args.warmup + i)
    core.sync()
    el = (time.perf_counter() - t0) / args.config4_steps
    core.close()
    return {"workload": f"config4 in-core: room {sc.tri_count} tris, {W4}x{H4} 1 spp, maxPathLength 4, one process, "
                        f"deviceCount {ndev} (band partition + xGMI peer-copy gather inside the core), RenderSystem's "
                        f"six Setting calls + Render per frame",
            "scaling": "strong", "n_gpus": ndev, "steps": args.config4_steps,
            "value": round((int(counts[0]) + int(counts[1])) / el / 1e6, 3), "unit": "Mrays/s (primary+secondary)",
            "ms_per_frame": round(el * 1e3, 4), "setup_s": round(setup, 2),
            "rays_per_frame": {"primary_plus_bounce1": int(counts[0]) + int(counts[1]),
                               "deeper": int(counts[2:16].sum()), "shadow": int(counts[16])}}


def roofline_of(core, sc, W, H, dev, kernel_iters):
    """The dominant kernel (bounce-ray closest hit, per-ray traversal) and the primary-ray launch, timed
    with their own HIP events; priced by the committed counter summaries of the same kernels."""
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
        ms = core.trace_closest_device(ro.data_ptr(), rd.data_ptr(), n, hits.data_ptr(), kernel_iters)
        core.setting("unitCoherent", 0)
        return ms, hits.cpu().numpy().view(np.uint32)

    ms_p, hits_p = launch(o4, d4, True)
    bo, bd = scene.bounce_rays(sc.meshes[0], o4, d4, hits_p)
    # the frame's shade writes them into two-ended segments (chordSplit): its trace takes them in this order
    order = scene.chord_order(bo, bd, *scene.mesh_box(sc.meshes[0]), core.get_setting("chordSplit"))
    bo, bd = np.ascontiguousarray(bo[order]), np.ascontiguousarray(bd[order])
    ms, _ = launch(bo, bd, False)
    n, n_p = len(bo), len(o4)
    version = int(core.get_setting("traceVersion"))
    kname = TRACE_KERNEL.get(version, f"traceVersion {version}")
    if version == 7:
        # the exact variant the unit launch runs (single instance, the unit queries' waves): its counter summaries only
        # (tools/pmc_round.sh names it with --kernel; round 5's names carried a third template argument, the W8 switch)
        kname = f"k_trace_closest4d<true, {int(core.get_setting('unitTraceWaves'))}"
    cyc, cyc_mix, cyc_src = valu_cycles_per_instruction()
    peak = SIMDS * CLOCK_GHZ / cyc                     # G wave64 VALU instructions / s
    peak_mix = SIMDS * CLOCK_GHZ / cyc_mix
    sq_src, sq = newest("*_pmc_trace_sq.json", lambda d: d.get("kernel", "").startswith(kname))
    tr_src, tr = newest("*_pmc_traffic.json", lambda d: d.get("kernel", "").startswith(kname))
    fix = json.load(open(ROOT / "tests" / "golden" / "config2_bounce_visits.json"))
    bpr = 32 + 20 + 32 * fix["mean_node_records"] + 36 * fix["mean_tri_tests"]
    model_gbs = bpr * n / (ms * 1e-3) / 1e9
    valu = sq["valu_wave_insts_per_launch"] if sq else None
    achieved = valu / (ms * 1e-3) / 1e9 if valu else None
    traffic = tr["bytes_per_launch"] if tr else None
    hbm_gbs = traffic / (ms * 1e-3) / 1e9 if traffic else None
    lanes = sq.get("valu_lane_utilisation") if sq else None
    frac = achieved / peak if achieved else None
    roof = {
        "bound": "valu", "achieved": round(achieved, 1) if achieved else None, "peak": round(peak, 1),
        "unit": "G wave64 VALU instructions/s", "frac": round(frac, 4) if frac else None,
        "traffic": traffic,
        # what the frac cannot hide.  Instructions per ray (a VALU roofline rewards issuing more of them) and
        # the frac times the lanes that do work in an instruction
        "valu_insts_per_ray": round(valu / n, 2) if valu else None,
        "useful_frac": round(frac * lanes, 4) if frac and lanes else None,
        "frac_vs_mix_peak": round(achieved / peak_mix, 4) if achieved else None, "mix_peak": round(peak_mix, 1),
        "kernel": f"{kname} (per-ray BVH4 traversal, traceVersion {version}, the core's default settings) on the "
                  f"frame's {n} diffuse bounce rays, in the frame's order (two-ended segments, chordSplit)",
        "kernel_ms": round(ms, 4), "rays_per_launch": n,
        "valu_insts_per_launch": valu, "valu_lane_utilisation": lanes,
        "peak_basis": f"{SIMDS} SIMDs x {CLOCK_GHZ} GHz / {cyc:.3f} cycles per wave64 VALU instruction: the fastest class measured, "
                      f"VOP2 v_add_f32 / v_mul_f32 at 8 waves per SIMD ({cyc_src or 'MI355X_MICROARCH.md: 2 (SIMD-32)'}); "
                      f"mix_peak: the node step's instruction mix, {cyc_mix:.3f} cycles",
        "evidence": {"sq": sq_src, "traffic": tr_src},
        "hbm": {"measured_GBs": round(hbm_gbs, 1) if hbm_gbs else None,
                "measured_frac": round(hbm_gbs / HBM_PEAK_GBS, 4) if hbm_gbs else None,
                "model_bytes_per_ray": round(bpr, 1), "model_GBs": round(model_gbs, 1),
                "model_frac": round(model_gbs / HBM_PEAK_GBS, 4),
                "model": "SURVEY §8(d): 32 ray + 20 hit + 32 x node records + 36 x triangle tests of the reference "
                         "BVH2 traversal (tests/golden/config2_bounce_visits.json); the BVH and triangles are "
                         "L2 / Infinity-Cache resident, so DRAM sees the measured bytes, not the model"},
    }
    psq_src, psq = newest("*_pmc_packet_sq.json")
    pvalu = psq["valu_wave_insts_per_launch"] if psq and "valu_wave_insts_per_launch" in psq else None
    prim = {"bound": "valu", "kernel": ("k_trace_closest_packet (wave-uniform packet traversal)"
                                        if core.get_setting("usePackets") else kname) + " on the 1080p primary rays",
            "kernel_ms": round(ms_p, 4), "rays_per_launch": n_p,
            "achieved": round(pvalu / (ms_p * 1e-3) / 1e9, 1) if pvalu else None, "peak": round(peak, 1),
            "frac": round(pvalu / (ms_p * 1e-3) / 1e9 / peak, 4) if pvalu else None, "evidence": psq_src}
    detail = {"trace_Mrays_s_bounce": round(n / (ms * 1e-3) / 1e6, 1),
              "trace_Mrays_s_primary": round(n_p / (ms_p * 1e-3) / 1e6, 1)}
    return roof, prim, detail, model_gbs


def roofline_config5(c5):
    """The HBM view of the DRAM-real workload (config 5: 1 GB of BVH + triangles, beyond the 256 MB Infinity Cache): the
    per-ray closest-hit launch's measured bytes (2 x FETCH_SIZE + WRITE_SIZE, separate --pmc passes over config-5
    frames, the committed *_pmc_config5_traffic.json) / its launch time in the same passes / 8 TB/s.  An UPPER bound of
    DRAM traffic: FETCH_SIZE also counts Infinity-Cache (MALL) hits (MI355X_MICROARCH.md, the HBM / rocprofv3 section).
    The live launch times of this run's config-5 frames (CoreStats traceTime0 / traceTime1: the primary and the bounce
    launch, each with its launch gap) sit beside it."""
    src, d = newest("*_pmc_config5_traffic.json")
    if not d:
        return None
    ks = [k for k in d["kernels"] if k["kernel"].startswith("void k_trace_closest4d")]
    if not ks:
        return None
    k = max(ks, key=lambda r: r["launch_ms_median"] * r["launches"])
    gbs = k["bytes_per_launch"] / (k["launch_ms_median"] * 1e-3) / 1e9
    out = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
           "traffic": k["bytes_per_launch"], "upper_bound": True,
           "kernel": k["kernel"].split("(")[0] + " (config 5: per-ray closest hit, primary and bounce launches of 1080p 8 spp frames)",
           "kernel_ms": k["launch_ms_median"], "launches": k["launches"], "evidence": src,
           "note": "bytes = 2 x FETCH_SIZE + WRITE_SIZE per launch (gfx950 calibration), medians over the passes' launches; "
                   "FETCH_SIZE counts Infinity-Cache hits too, so frac is an upper bound of the DRAM fraction"}
    if c5:
        cs = c5["coreStats_ms"]
        out["live_launch_ms"] = {"primary": cs["trace0"], "bounce": cs["trace1"]}
    # the other side of the bracket.  The unique node / triangle records one closest-hit launch reads (LH2_TOUCH
    # build, *_config5_touch.json) plus its ray and hit streams, less what the 256 MiB Infinity Cache and the L2s can hold from
    # before the launch, must cross the HBM interface at least once: a LOWER bound of its DRAM bytes.  Priced over this run's
    # live primary and bounce launch times (CoreStats, each with its launch gap)
    tsrc, t = newest("*_config5_touch.json")
    if t and c5:
        lb = {l["kind"]: l for l in t["launches"]}
        cs = c5["coreStats_ms"]
        if "primary" in lb and "bounce" in lb and cs["trace0"] > 0 and cs["trace1"] > 0:
            lo_bytes = lb["primary"]["dram_lower_bound_bytes"] + lb["bounce"]["dram_lower_bound_bytes"]
            lo_gbs = lo_bytes / ((cs["trace0"] + cs["trace1"]) * 1e-3) / 1e9
            out["lower_bound"] = {"achieved": round(lo_gbs, 1), "frac": round(lo_gbs / HBM_PEAK_GBS, 4), "bytes_per_frame": lo_bytes,
                                  "unique_bytes": {k: lb[k]["unique_bytes"] for k in ("primary", "bounce")},
                                  "evidence": tsrc,
                                  "note": "max(0, unique bytes - 288 MiB) per launch (tools/touch_summary.py) over the live "
                                          "primary + bounce launch times; the DRAM fraction lies between frac_lower and frac"}
            out["frac_lower"] = out["lower_bound"]["frac"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--tris", type=int, default=100_000)
    ap.add_argument("--room-tris", type=int, default=1_000_000)
    ap.add_argument("--config4-steps", type=int, default=10)
    ap.add_argument("--no-config4", action="store_true")
    ap.add_argument("--config-steps", type=int, default=10, help="frames timed for configs 3 and 5")
    ap.add_argument("--no-configs", action="store_true", help="skip configs 3, 5 and config4_incore")
    ap.add_argument("--no-config5", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--setting", action="append", default=[], help="name=value core setting before loading (A/B runs)")
    args = ap.parse_args()

    # provenance: the library must be built from the checked-out sources (lh2_version() "srchash=")
    want, got = build_info.source_hash(), build_info.library_hash()
    if want != got:
        raise SystemExit(f"libRenderCore_MI355X.so srchash={got} but the sources hash to {want}: rebuild it")

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
    gather = TileGather(rank, world, W, H, dev)
    assert core.tile_rows() == gather.rows
    elapsed, tot, counts = timed_frames(core, sc, gather, args.steps, args.warmup, world, dev)
    st = core.stats()
    rays_total = tot[0]
    value = rays_total * args.steps / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3

    out = None
    if rank == 0:
        roof, prim, det, model_gbs = roofline_of(core, sc, W, H, dev, args.kernel_iters)
        # the per-ray byte model of the kernels timed in a step must fit the step at HBM peak (the packet
        # kernel fetches each node once per 64 rays, so it is priced by its VALU issue, not this model)
        step_model_gbs = model_gbs * roof["kernel_ms"] / ms_step
        assert step_model_gbs <= HBM_PEAK_GBS, ("byte model exceeds HBM peak over the step", step_model_gbs)
        roof["hbm"]["model_GBs_over_step"] = round(step_model_gbs, 1)
        info = core.scene_info()
        out = {
            "metric": "Mrays/s (primary+secondary) at 1080p 1spp",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"config2: {args.tris} random tris (xorshift32 0x12345678), {W}x{H} frame "
                                   f"({args.width}x{args.height} paths per GPU, {BAND}-row bands), 1 spp, "
                                   f"full wavefront frame (primary + bounce-1 rays); strong scaling of config 4 "
                                   f"(4K, frame split across the GPUs) in 'config4'",
                       "frame": [W, H], "spp": 1, "tris": args.tris, "parallelism": f"tiles{world}",
                       "frames": "a still camera converging: one Restart, then Converge (new samples every step)"},
            "roofline": roof,
            "roofline_primary": prim,
            "detail": {"primary_rays": int(counts[0]), "secondary_rays": int(counts[1]),
                       "deep_rays": int(counts[2:16].sum()), "shadow_rays": int(counts[16]), **det,
                       "trace_Mrays_s_frame": round(rays_total / world / ((st.traceTime0 + st.traceTime1) * 1e6), 1)
                       if st.traceTime0 + st.traceTime1 > 0 else None,
                       "traceTime0_ms": round(st.traceTime0 * 1e3, 4), "traceTime1_ms": round(st.traceTime1 * 1e3, 4),
                       "shadeTime_ms": round(st.shadeTime * 1e3, 4), "bvh_nodes": info["nodes"],
                       "bvh_depth": info["max_depth"], "setup_s": round(build_s, 3)},
            "build": {"srchash": got, "lh2_version": core.lib.lh2_version().decode()},
        }
    core.close()
    c4 = None if args.no_config4 else config4(args, rank, world, local, dev)
    c4in = c3 = c5 = c2r = None
    if not args.no_configs:
        # the in-core multi-device run uses the node's first `world` GPUs from rank 0 alone: the other ranks
        # wait at a host-side (gloo) barrier, so no collective kernel occupies their GPUs meanwhile
        host = dist.new_group(backend="gloo") if world > 1 else None
        if world > 1:
            dist.barrier(group=host)
        if rank == 0:
            c4in = config4_incore(args, world)
            if world == 1:
                c2r = config2_restart(args, local)
                c3 = config3(args, local)
                c5 = None if args.no_config5 else config5(args, local)
        if world > 1:
            dist.barrier(group=host)
    if rank == 0:
        out["config2_restart"] = c2r
        out["config4"] = c4
        out["config4_incore"] = c4in
        out["config3"] = c3
        out["config5"] = c5
        out["roofline_config5"] = roofline_config5(c5) if world == 1 else None
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(sc, args.width, args.height, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
