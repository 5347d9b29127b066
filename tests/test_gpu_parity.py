"""GPU parity tests: the HIP render core (through the C-ABI) against the CPU oracle.

Bar (BASELINE.md "Parity"): bit-exact primary rays and hit records
{t, triid, instid, uv16}; identical occlusion bits; identical per-bounce ray counts; accumulator
relative L2 <= 1e-4 (north_star tolerance; only the float atomic summation order differs)."""
import numpy as np
import pytest

from lighthouse2_amd import abi, scene
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

REL_L2_TOL = 1e-4


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _load_both(core, sc, w, h, spp=1):
    sc.load_into(core)
    core.set_target(w, h, spp)
    o = Oracle()
    sc.load_into(o)
    o.set_target(w, h, spp)
    return o


def test_native_library_is_loaded(core):
    maps = open("/proc/self/maps").read()
    assert "libRenderCore_MI355X.so" in maps
    assert core.stats().SMcount >= 1


@pytest.mark.parametrize("pass_,spp", [(0, 1), (0, 2), (300, 1)])
def test_camera_rays_bitexact(core, pass_, spp):
    w, h = 96, 54
    sc = scene.config2_scene(n=2000, width=w, height=h)
    sc.view = scene.camera_view((0.3, 0.2, -12), (0.05, -0.02, 1), fov_deg=50, aspect=w / h, aperture=0.05,
                                distortion=0.0 if pass_ == 0 else 0.05, pixel_height=h)
    o = _load_both(core, sc, w, h, spp)
    o.setting("epsilon", 1e-4)
    core.setting("epsilon", 1e-4)
    R0 = 0x9E3779B9
    go, gd, gs = core.generate_eye_rays(sc.view, R0, pass_)
    oo, od, os_ = o.generate_eye_rays(sc.view, R0, pass_)
    assert np.array_equal(go.view(np.uint32), oo.view(np.uint32))
    assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))
    assert np.array_equal(gs.view(np.uint32), os_.view(np.uint32))


def _random_rays(n, seed, center=(0, 0, 0), radius=14.0, tmin=1e-4):
    rng = np.random.default_rng(seed)
    o = rng.normal(size=(n, 3)).astype(np.float32)
    o = o / np.linalg.norm(o, axis=1, keepdims=True) * np.float32(radius) + np.array(center, np.float32)
    tgt = rng.uniform(-4, 4, size=(n, 3)).astype(np.float32)
    d = tgt - o
    d = (d * (np.float32(1) / np.sqrt((d * d).sum(1, dtype=np.float32)))[:, None]).astype(np.float32)
    O4 = np.concatenate([o, np.full((n, 1), tmin, np.float32)], 1)
    D4 = np.concatenate([d, np.full((n, 1), 1e34, np.float32)], 1)
    return O4, D4


def test_trace_closest_bitexact_random_tris(core):
    w, h = 160, 90
    sc = scene.config2_scene(n=20000, width=w, height=h)
    o = _load_both(core, sc, w, h)
    O4, D4 = _random_rays(50000, 1)
    hg = core.trace_closest(O4, D4)
    ho = o.trace_closest(O4, D4)
    assert (ho[:, 1] != 0xFFFFFFFF).mean() > 0.3
    assert np.array_equal(hg, ho), np.argwhere((hg != ho).any(1))[:10]


def test_trace_closest_primary_rays_bitexact(core):
    w, h = 192, 108
    sc = scene.config2_scene(n=20000, width=w, height=h)
    o = _load_both(core, sc, w, h)
    core.setting("epsilon", 1e-4)
    o.setting("epsilon", 1e-4)
    O4, D4, _ = o.generate_eye_rays(sc.view, 0, 0)
    assert np.array_equal(core.trace_closest(O4, D4), o.trace_closest(O4, D4))


def test_trace_closest_instanced_transformed(core):
    sc = scene.instanced_scene(meshes=6, tris_per_mesh=3000, width=64, height=36, grid=3, spacing=12.0)
    scene.animate_instances(sc, 3)
    # non-uniform scale + shear on one instance: the ray is transformed without renormalisation
    T = sc.instances[2][1].copy()
    T[0, 0] *= 1.7
    T[1, 0] += 0.3
    sc.instances[2] = (2, T)
    o = _load_both(core, sc, 64, 36)
    O4, D4 = _random_rays(40000, 2, center=(0, 0, 0), radius=40.0)
    rng = np.random.default_rng(3)
    tgt = np.concatenate([rng.uniform(-20, 20, (40000, 1)), rng.uniform(-4, 4, (40000, 1)), rng.uniform(-20, 20, (40000, 1))], 1)
    d = (tgt - O4[:, :3]).astype(np.float32)
    D4[:, :3] = d / np.linalg.norm(d, axis=1, keepdims=True)
    hg = core.trace_closest(O4, D4)
    ho = o.trace_closest(O4, D4)
    assert (ho[:, 1] != 0xFFFFFFFF).mean() > 0.05
    assert np.array_equal(hg, ho), np.argwhere((hg != ho).any(1))[:10]


def test_trace_any_matches(core):
    sc = scene.config2_scene(n=20000, width=64, height=36)
    o = _load_both(core, sc, 64, 36)
    O4, D4 = _random_rays(30001, 4, tmin=0.0)
    rng = np.random.default_rng(5)
    D4[:, 3] = rng.uniform(1.0, 20.0, len(D4)).astype(np.float32)   # finite tmax, like shadow rays
    mg = core.trace_any(O4, D4)
    mo = o.trace_any(O4, D4)
    assert 0.05 < np.unpackbits(mo.view(np.uint8)).mean() < 0.95
    assert np.array_equal(mg, mo)


@pytest.mark.parametrize("name", ["config2_light", "room"])
def test_render_frame_parity(core, name):
    w, h = 160, 90
    if name == "room":
        sc = scene.room_scene(30000, w, h)
    else:
        sc = scene.config2_scene(n=20000, width=w, height=h, sky=True, light=True)
    o = _load_both(core, sc, w, h)
    core.set_probe(w // 2, h // 2)
    o.set_probe(w // 2, h // 2)
    sc.render_frame(core)
    sc.render_frame(o)
    cg, co = core.ray_counts(), o.ray_counts()
    assert np.array_equal(cg, co), (cg, co)
    ag, ao = core.accumulator(), o.accumulator()
    assert rel_l2(ag[..., :3], ao[..., :3]) <= REL_L2_TOL
    assert rel_l2(ag[..., 3], ao[..., 3]) <= 1e-6
    st, ost = core.stats(), o.stats()
    assert (st.probedTriid, st.probedInstid) == (ost.probedTriid, ost.probedInstid)
    assert st.primaryRayCount == co[0] and st.bounce1RayCount == co[1]


def test_converging_frames_and_spp(core):
    w, h = 96, 54
    sc = scene.room_scene(20000, w, h)
    o = _load_both(core, sc, w, h, spp=2)
    for f in range(3):
        conv = 1 if f == 0 else 0
        sc.render_frame(core, converge=conv)
        sc.render_frame(o, converge=conv)
        assert np.array_equal(core.ray_counts(), o.ray_counts())
    ag, ao = core.accumulator(), o.accumulator()
    assert rel_l2(ag[..., :3], ao[..., :3]) <= REL_L2_TOL
    assert rel_l2(core.frame()[..., :3], o.frame()[..., :3]) <= REL_L2_TOL


def test_tile_partition_invariance(core):
    """Rendering the frame as row tiles (the multi-GPU partition) gives the untiled result."""
    w, h = 128, 72
    sc = scene.room_scene(20000, w, h)
    sc.load_into(core)
    core.set_target(w, h, 1)
    sc.render_frame(core)
    full = core.accumulator()
    parts = np.zeros_like(full)
    for y0, y1 in ((0, 30), (30, 31), (31, 72)):
        core.set_target(w, h, 1)
        core.set_tile(y0, y1)
        sc.render_frame(core)
        parts[y0:y1] = core.accumulator()[y0:y1]
    core.set_tile(0, -1)
    assert rel_l2(parts[..., :3], full[..., :3]) <= 1e-6


def test_band_partition_matches_full_frame(core):
    """The N-GPU partition (8-row bands round-robin, packed by lh2_core_pack_tile) rendered rank by rank
    on one GPU and reassembled equals the untiled frame."""
    import torch
    from lighthouse2_amd import parallel
    w, h, world = 96, 60, 3
    sc = scene.room_scene(20000, w, h)
    sc.load_into(core)
    core.set_target(w, h, 1)
    core.set_tile(0, -1)
    sc.render_frame(core)
    full = core.accumulator()
    full_frame = core.frame()
    tiles = []
    for r in range(world):
        core.set_target(w, h, 1)
        core.set_tile_bands(r, world, parallel.BAND)
        sc.render_frame(core)
        rows = core.tile_rows()
        assert rows == len(parallel.band_rows(r, world, h))
        # the rank finalizes its own rows (k_finalize's row map): they equal the untiled frame's
        own = np.asarray(parallel.band_rows(r, world, h))
        assert rel_l2(core.frame()[own][..., :3], full_frame[own][..., :3]) <= 1e-6
        t = torch.empty((rows, w, 4), dtype=torch.float32, device="cuda")
        core.pack_tile(t.data_ptr())
        tiles.append(t.cpu().numpy())
    core.set_tile(0, -1)
    frame = parallel.assemble(tiles, world, h)
    assert rel_l2(frame[..., :3], full[..., :3]) <= 1e-6
    assert np.array_equal(frame[..., 3], full[..., 3])


def test_instanced_animated_frames_parity(core):
    """Config 5 in miniature: several instanced meshes, new instance transforms every frame
    (SetInstance + UpdateToplevel), 2 spp, converging frames."""
    w, h = 96, 54
    sc = scene.instanced_scene(meshes=4, tris_per_mesh=3000, width=w, height=h, grid=2, spacing=12.0)
    sc.view = scene.camera_view((0, 6, -12), (0, -0.3, 1), fov_deg=60, aspect=w / h, pixel_height=h)
    o = _load_both(core, sc, w, h, spp=2)
    for f in range(3):
        scene.animate_instances(sc, f)
        for tgt in (core, o):
            for k, (mesh, T) in enumerate(sc.instances):
                tgt.set_instance(k, mesh, T)
            tgt.update_toplevel()
        sc.render_frame(core, converge=1 if f == 0 else 0)
        sc.render_frame(o, converge=1 if f == 0 else 0)
        assert np.array_equal(core.ray_counts(), o.ray_counts())
    ag, ao = core.accumulator(), o.accumulator()
    assert rel_l2(ag[..., :3], ao[..., :3]) <= REL_L2_TOL


def test_room_depth4_parity(core):
    """Config 3 in miniature: the procedural room (specular chains, glass, smooth spheres, two area
    lights) with maxPathLength 4."""
    w, h = 128, 72
    sc = scene.room_scene(40000, w, h)
    o = _load_both(core, sc, w, h)
    for tgt in (core, o):
        tgt.setting("maxPathLength", 4)
    sc.render_frame(core)
    sc.render_frame(o)
    cg, co = core.ray_counts(), o.ray_counts()
    assert np.array_equal(cg, co), (cg, co)
    assert co[4] == 0 and co[3] > 0                 # bounded at 4 vertices, specular chains reach it
    ag, ao = core.accumulator(), o.accumulator()
    assert rel_l2(ag[..., :3], ao[..., :3]) <= REL_L2_TOL
    core.setting("maxPathLength", 16)


@pytest.mark.parametrize("kind", ["random", "primary", "instanced"])
def test_packet_traversal_bitexact(fresh_core, kind):
    """Packet traversal (wave-uniform path for 64 rays over the BVH2, lh2_trace_packet.inc) gives every
    ray exactly the per-ray traversal's hit record, also for incoherent rays and through instances."""
    if kind == "instanced":
        sc = scene.instanced_scene(meshes=6, tris_per_mesh=3000, width=64, height=36, grid=3, spacing=12.0)
        scene.animate_instances(sc, 2)
    else:
        sc = scene.config2_scene(n=20000, width=192, height=108)
    o = _load_both(fresh_core, sc, 192, 108)
    fresh_core.setting("epsilon", 1e-4)
    o.setting("epsilon", 1e-4)
    if kind == "primary":
        O4, D4, _ = o.generate_eye_rays(sc.view, 0, 0)
        perm = scene.tiled_order(192, 108)
        O4, D4 = np.ascontiguousarray(O4[perm]), np.ascontiguousarray(D4[perm])
    else:
        O4, D4 = _random_rays(30001, 7, radius=40.0 if kind == "instanced" else 14.0)
    fresh_core.setting("packetPrimary", 1)
    fresh_core.setting("unitCoherent", 1)
    hp = fresh_core.trace_closest(O4, D4)
    fresh_core.setting("unitCoherent", 0)
    ho = o.trace_closest(O4, D4)
    assert (ho[:, 1] != 0xFFFFFFFF).mean() > 0.05
    assert np.array_equal(hp, ho), np.argwhere((hp != ho).any(1))[:10]


@pytest.mark.parametrize("version,leaf_batch,max_leaf", [(1, 0, 2), (1, 16, 2), (1, 8, 4), (7, 0, 1), (7, 1, 2), (7, 6, 1), (7, 32, 1),
                                                       (7, 8, 4), (7, 64, 2)])
def test_traversal_variants_bitexact(fresh_core, version, leaf_batch, max_leaf):
    """Both per-ray traversal loops (the reference BVH2 loop trace_stream, and the BVH4 loop of
    lh2_trace4d.inc with its leaf slot), with and without leaf parking / batching, over trees of
    different leaf sizes, return the oracle's hit records and occlusion bits: hits do not depend on the
    tree or the visiting order."""
    fresh_core.setting("bvhMaxLeaf", max_leaf)
    fresh_core.setting("traceVersion", version)
    fresh_core.setting("leafBatch", leaf_batch)
    sc = scene.instanced_scene(meshes=4, tris_per_mesh=4000, width=64, height=36, grid=2, spacing=10.0)
    scene.animate_instances(sc, 1)
    o = _load_both(fresh_core, sc, 64, 36)
    O4, D4 = _random_rays(30001, 11, radius=30.0)
    hg = fresh_core.trace_closest(O4, D4)
    ho = o.trace_closest(O4, D4)
    assert (ho[:, 1] != 0xFFFFFFFF).mean() > 0.05
    assert np.array_equal(hg, ho), np.argwhere((hg != ho).any(1))[:10]
    D4[:, 3] = np.random.default_rng(12).uniform(1.0, 40.0, len(D4)).astype(np.float32)
    assert np.array_equal(fresh_core.trace_any(O4, D4), o.trace_any(O4, D4))


@pytest.mark.parametrize("version,max_leaf,alpha,budget", [(7, 1, 1e-5, 1.0), (7, 4, 1e-5, 1.0), (7, 2, 1e-5, 1.0),
                                                            (1, 2, 1e-5, 1.0), (7, 1, 1e-7, 1.0), (7, 1, 0.0, 1.0),
                                                            (7, 1, 1e-7, 0.002)])
def test_spatial_splits_bitexact(fresh_core, version, max_leaf, alpha, budget):
    """Spatial splits (bvhSpatial, the default: SBVH references, a triangle in several leaves with
    clipped boxes; 0 = object splits only) change the tree only: closest hits, occlusion and a
    packet-traced frame equal the oracle's.  A small bvhSpatialBudget runs the duplication budget dry
    (splits abandoned and reservations returned part-way through the build)."""
    fresh_core.setting("bvhSpatial", alpha)
    fresh_core.setting("bvhSpatialBudget", budget)
    fresh_core.setting("bvhMaxLeaf", max_leaf)
    fresh_core.setting("traceVersion", version)
    sc = scene.config2_scene(n=20000, width=64, height=36)
    o = _load_both(fresh_core, sc, 64, 36)
    assert fresh_core.get_setting("bvhSpatial") == np.float32(alpha)
    O4, D4 = _random_rays(30001, 21, radius=8.0)
    hg, ho = fresh_core.trace_closest(O4, D4), o.trace_closest(O4, D4)
    assert (ho[:, 1] != 0xFFFFFFFF).mean() > 0.3
    assert np.array_equal(hg, ho), np.argwhere((hg != ho).any(1))[:10]
    D4[:, 3] = np.random.default_rng(22).uniform(0.5, 20.0, len(D4)).astype(np.float32)
    assert np.array_equal(fresh_core.trace_any(O4, D4), o.trace_any(O4, D4))
    sc.render_frame(fresh_core)
    sc.render_frame(o)
    assert np.array_equal(fresh_core.ray_counts(), o.ray_counts())
    assert rel_l2(fresh_core.accumulator()[..., :3], o.accumulator()[..., :3]) <= REL_L2_TOL


@pytest.mark.parametrize("collapse,max_leaf", [(1, 1), (1, 2), (1, 4), (0, 1), (0, 3)])
def test_bvh4_collapse_bitexact(fresh_core, collapse, max_leaf):
    """The BVH4 collapses (bvh4Collapse 1: dynamic programming, 0: greedy) of SBVH trees with leaves of up
    to max_leaf triangles, with instances: hits, occlusion and a frame equal the oracle's."""
    fresh_core.setting("bvh4Collapse", collapse)
    fresh_core.setting("bvhMaxLeaf", max_leaf)
    sc = scene.instanced_scene(meshes=3, tris_per_mesh=6000, width=64, height=36, grid=2, spacing=10.0)
    scene.animate_instances(sc, 1)
    o = _load_both(fresh_core, sc, 64, 36)
    O4, D4 = _random_rays(30001, 31, radius=30.0)
    hg, ho = fresh_core.trace_closest(O4, D4), o.trace_closest(O4, D4)
    assert (ho[:, 1] != 0xFFFFFFFF).mean() > 0.05
    assert np.array_equal(hg, ho), np.argwhere((hg != ho).any(1))[:10]
    D4[:, 3] = np.random.default_rng(32).uniform(1.0, 40.0, len(D4)).astype(np.float32)
    assert np.array_equal(fresh_core.trace_any(O4, D4), o.trace_any(O4, D4))
    sc.render_frame(fresh_core)
    sc.render_frame(o)
    assert np.array_equal(fresh_core.ray_counts(), o.ray_counts())
    assert rel_l2(fresh_core.accumulator()[..., :3], o.accumulator()[..., :3]) <= REL_L2_TOL


@pytest.mark.parametrize("version,waves", [(1, 8), (7, 8), (7, 7)])
def test_bvh4_deep_stack(fresh_core, version, waves):
    """A deep BLAS (triangles shrinking geometrically along a line: a chain-like SAH tree) next to the
    random cloud: BVH4 nodes push up to three children per level, the LDS part of the traversal
    stack spills into the global part, and hits stay exact; with the closest-hit kernel's 8-wave
    variant (64 VGPRs, 8 blocks per CU) and its 7-wave one (traceWaves / unitTraceWaves)."""
    k = np.arange(120, dtype=np.float32)
    x = (6.0 * 0.93 ** k).astype(np.float32)
    s_ = (0.02 * 0.93 ** k).astype(np.float32)
    z0 = np.zeros_like(x)
    v0 = np.stack([x, -s_, z0], 1)
    v1 = np.stack([x + s_, s_, z0], 1)
    v2 = np.stack([x - s_, s_, s_], 1)
    chain = abi.tris_from_vertices(v0, v1, v2, 0)
    sc = scene.config2_scene(n=5000, width=64, height=36)
    sc.meshes.append(chain)
    sc.instances.append((1, np.eye(4, dtype=np.float32)))
    fresh_core.setting("traceVersion", version)
    fresh_core.setting("traceWaves", waves)
    fresh_core.setting("unitTraceWaves", waves)      # the unit queries below launch this variant
    assert fresh_core.get_setting("traceBlocksPerCU") == waves
    o = _load_both(fresh_core, sc, 64, 36)
    info = fresh_core.scene_info()
    assert info["max_depth"] >= 14, info
    O4, D4 = _random_rays(20001, 13)
    # half of the rays aimed at chain triangles (their centroids), from random directions
    rng = np.random.default_rng(14)
    j = rng.integers(0, len(x), 10000)
    tgt = ((v0[j] + v1[j] + v2[j]) / 3).astype(np.float32)
    d = tgt - O4[:10000, :3]
    D4[:10000, :3] = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    hg, ho = fresh_core.trace_closest(O4, D4), o.trace_closest(O4, D4)
    assert (ho[:10000, 2] == 1).mean() > 0.2   # instance 1 (the chain) is hit
    assert np.array_equal(hg, ho), np.argwhere((hg != ho).any(1))[:10]
    D4[:, 3] = np.random.default_rng(15).uniform(1.0, 20.0, len(D4)).astype(np.float32)
    assert np.array_equal(fresh_core.trace_any(O4, D4), o.trace_any(O4, D4))


@pytest.mark.parametrize("kind", ["diffuse", "emissive", "specular"])
def test_terminal_shade_frame_parity(fresh_core, kind):
    """Scenes without lights (the bench's config 2): the last shade pass drops hits that cannot
    contribute (ShadeParams::terminal).  With an emissive quad but no light list the core must keep
    shading them (its colour > 1 makes them emit).  With every other triangle a mirror, paths go on
    past their second vertex, so the drop runs in mid-path shade passes (k_shade<true>) as well as in
    the last one (k_shade_last).  Oracle parity, and the same frame with the drop switched off
    matches to float-summation order."""
    w, h = 160, 90
    sc = scene.config2_scene(n=20000, width=w, height=h, sky=True, light=kind == "emissive")
    sc.area_lights = []
    if kind == "specular":
        sc.materials.append(abi.make_material((0.9, 0.9, 0.9), roughness=0.0))
        sc.meshes[0].view(np.uint32)[::2, abi.TRI["material"]] = 1
    o = _load_both(fresh_core, sc, w, h)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", 5)
    sc.render_frame(fresh_core)
    sc.render_frame(o)
    cg, co = fresh_core.ray_counts(), o.ray_counts()
    assert np.array_equal(cg, co), (cg, co)
    assert co[1] > 0 and (kind != "specular" or co[3] > 0), co
    ag, ao = fresh_core.accumulator(), o.accumulator()
    assert rel_l2(ag[..., :3], ao[..., :3]) <= REL_L2_TOL
    assert rel_l2(ag[..., 3], ao[..., 3]) <= 1e-6
    fresh_core.setting("terminalShade", 0)
    sc.render_frame(fresh_core)
    a0 = fresh_core.accumulator()
    fresh_core.setting("terminalShade", 1)
    assert rel_l2(ag[..., :3], a0[..., :3]) <= 1e-6
    assert np.array_equal(ag[..., 3], a0[..., 3])


@pytest.mark.parametrize("version", [1, 7])
@pytest.mark.parametrize("start", [0, 1])
def test_single_instance_start_bitexact(fresh_core, version, start):
    """One instance (sheared and scaled): with singleInstanceStart the rays begin at its TLAS leaf
    instead of the TLAS root; per-ray (BVH2 / BVH4) and packet hits match the oracle bit for bit."""
    sc = scene.config2_scene(n=20000, width=64, height=36)
    T = np.eye(4, dtype=np.float32)
    T[0, 0], T[1, 0], T[2, 3] = 1.7, 0.3, 2.0
    sc.instances[0] = (0, T)
    fresh_core.setting("singleInstanceStart", start)
    fresh_core.setting("traceVersion", version)
    o = _load_both(fresh_core, sc, 64, 36)
    O4, D4 = _random_rays(50000, 11, radius=16.0)
    hg, ho = fresh_core.trace_closest(O4, D4), o.trace_closest(O4, D4)
    assert 0.05 < (ho[:, 1] != 0xFFFFFFFF).mean() < 0.95
    assert np.array_equal(hg, ho), np.argwhere((hg != ho).any(1))[:10]
    D4[:, 3] = np.random.default_rng(4).uniform(1.0, 20.0, len(D4)).astype(np.float32)
    assert np.array_equal(fresh_core.trace_any(O4, D4), o.trace_any(O4, D4))
    if version == 7:
        fresh_core.setting("epsilon", 1e-4)
        o.setting("epsilon", 1e-4)
        sc.render_frame(fresh_core)
        sc.render_frame(o)
        assert np.array_equal(fresh_core.ray_counts(), o.ray_counts())


def test_no_lights_rng_stream_past_sample_256(fresh_core):
    """Without lights the shade kernel compiles NEE out (k_shade<*, NL>) but still draws its two random
    numbers past sample 1: from sample 256 on the BSDF sample uses the same seed's later draws, so
    a missing draw would change every extension direction there."""
    w, h, spp = 16, 9, 260
    sc = scene.config2_scene(n=20000, width=w, height=h, sky=True)
    sc.materials.append(abi.make_material((0.9, 0.9, 0.9), roughness=0.0))
    sc.meshes[0].view(np.uint32)[::2, abi.TRI["material"]] = 1
    o = _load_both(fresh_core, sc, w, h, spp=spp)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", 4)
    sc.render_frame(fresh_core)
    sc.render_frame(o)
    cg, co = fresh_core.ray_counts(), o.ray_counts()
    assert np.array_equal(cg, co), (cg, co)
    ag, ao = fresh_core.accumulator(), o.accumulator()
    assert rel_l2(ag[..., :3], ao[..., :3]) <= REL_L2_TOL


@pytest.mark.parametrize("version", [1, 7])
def test_lit_room_frame_traversal_versions(fresh_core, version):
    """The whole lit frame (closest hits of every bounce, any-hit shadow rays with the fused connect)
    through either per-ray loop: identical ray counts and accumulator."""
    w, h = 128, 72
    sc = scene.room_scene(40000, w, h)
    fresh_core.setting("traceVersion", version)
    o = _load_both(fresh_core, sc, w, h)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", 4)
    sc.render_frame(fresh_core)
    sc.render_frame(o)
    assert np.array_equal(fresh_core.ray_counts(), o.ray_counts())
    ag, ao = fresh_core.accumulator(), o.accumulator()
    assert rel_l2(ag[..., :3], ao[..., :3]) <= REL_L2_TOL


def _grazing_scene():
    """Two light-like quads at y = 15.95 (the room's lights, tessellated by the SBVH's spatial splits too) among
    a few thousand random triangles, far from the coordinate origin."""
    sc = scene.config2_scene(n=4000, width=64, height=36)
    tris = sc.meshes[0].copy()
    tris[:, 32:35] += np.float32(8.0)
    tris[:, 36:39] += np.float32(8.0)
    tris[:, 40:43] += np.float32(8.0)
    q1 = scene.quad_tris((0, -1, 0), (-8, 15.95, 0), 4, 4, 0)
    q2 = scene.quad_tris((0, -1, 0), (8, 15.95, 0), 4, 4, 0)
    sc.meshes[0] = np.concatenate([tris, q1, q2])
    return sc


def _grazing_rays(n, seed):
    """Shadow-ray-like queries from points just below the quads' plane (|y| ~ 16, so -o / d is large) to random
    points on a quad, at grazing angles; tmax within 2e-6 relative of the distance, so the quad's triangle lies
    just inside or just outside [tmin, tmax] (the room's light samples: SafeOrigin moves the origin, and a
    grazing ray meets the light's plane a little before distance - 2 epsilon, pathtracer.h:203-204)."""
    rng = np.random.default_rng(seed)
    o = np.stack([rng.uniform(-19, 19, n), 15.95 - rng.uniform(1e-3, 0.2, n), rng.uniform(-11.9, 11.9, n)], 1).astype(np.float32)
    side = np.where(rng.uniform(size=n) < 0.5, -8.0, 8.0)
    p = np.stack([side + rng.uniform(-2, 2, n), np.full(n, 15.95), rng.uniform(-2, 2, n)], 1).astype(np.float32)
    L = p - o
    dist = np.sqrt((L * L).sum(1, dtype=np.float32)).astype(np.float32)
    d = (L * (np.float32(1) / dist)[:, None]).astype(np.float32)
    O4 = np.concatenate([o, np.zeros((n, 1), np.float32)], 1)
    tmax = (dist * (1 + rng.uniform(-2e-6, 2e-6, n))).astype(np.float32)
    D4 = np.concatenate([d, tmax[:, None]], 1)
    return O4, D4


@pytest.mark.parametrize("version", [1, 7])
def test_grazing_rays_box_rounding(fresh_core, version):
    """Rays nearly parallel to a plane close to their origin's coordinate (shadow rays grazing the room's light
    quads): the slab distance (pl - o) / d is small while -o / d is large, so the rounding of the per-ray offset
    is an absolute error the boxes' relative pad does not cover; the offsets are rounded outward per axis
    (lh2_box4.inc slab_offsets).  Occlusion and closest hits, per-ray loops and packets, equal the oracle's,
    which tests (pl - o) * (1 / d) (RenderCore_Bart bvh.cpp:7-42).  Config 3 at 1080p lost 10 light samples to
    this before (tools/residual_config3.py)."""
    sc = _grazing_scene()
    fresh_core.setting("traceVersion", version)
    o = _load_both(fresh_core, sc, 64, 36)
    O4, D4 = _grazing_rays(60000, 41)
    og, oo = fresh_core.trace_any(O4, D4), o.trace_any(O4, D4)
    bits = np.unpackbits(oo.view(np.uint8), bitorder="little")[:len(O4)]
    assert 0 < bits.sum() < len(O4)
    assert np.array_equal(og, oo), np.nonzero(np.unpackbits((og ^ oo).view(np.uint8), bitorder="little"))[0][:10]
    D4[:, 3] = 1e34
    hg, ho = fresh_core.trace_closest(O4, D4), o.trace_closest(O4, D4)
    assert np.array_equal(hg, ho), np.argwhere((hg != ho).any(1))[:10]
    fresh_core.setting("packetPrimary", 1)
    fresh_core.setting("unitCoherent", 1)
    hp = fresh_core.trace_closest(O4, D4)
    fresh_core.setting("unitCoherent", 0)
    assert np.array_equal(hp, ho), np.argwhere((hp != ho).any(1))[:10]


def test_quantized_nodes_hold_the_f32_boxes(fresh_core):
    """k_quantize4 (bvh_gpu.hip): every child box of every BVH4 node (BLAS and TLAS, a mesh far from the origin
    and a chain of tiny triangles among them) is inside its quantized box in exact arithmetic, an empty slot is
    the inverted box with the pop marker as its reference, and the references are the f32 node's."""
    k = np.arange(60, dtype=np.float32)
    x = (6.0 * 0.9 ** k).astype(np.float32)
    s_ = (0.02 * 0.9 ** k).astype(np.float32)
    z0 = np.zeros_like(x)
    chain = abi.tris_from_vertices(np.stack([x, -s_, z0], 1), np.stack([x + s_, s_, z0], 1), np.stack([x - s_, s_, s_], 1), 0)
    sc = scene.config2_scene(n=4000, width=64, height=36)
    sc.meshes.append(chain)
    far = np.eye(4, dtype=np.float32)
    far[:3, 3] = (1000.0, -500.0, 250.0)
    sc.instances.append((1, far))
    sc.instances.append((0, far))
    sc.load_into(fresh_core)
    fresh_core.set_target(64, 36, 1)
    f, q = fresh_core.debug_bvh4()
    assert len(f) > 100
    lo = np.stack([f[:, 0:4], f[:, 8:12], f[:, 16:20]], 1).astype(np.float64)    # (n, axis, child)
    hi = np.stack([f[:, 4:8], f[:, 12:16], f[:, 20:24]], 1).astype(np.float64)
    valid = (np.isfinite(lo) & np.isfinite(hi) & (lo <= hi)).all(1)              # (n, child)
    origin = q[:, 0:3].view(np.float32).astype(np.float64)
    step = q[:, [3, 10, 11]].view(np.float32).astype(np.float64)                  # (n, axis): the grid steps 2^e
    assert np.all(np.frexp(step)[0] == 0.5)                                        # powers of two
    shifts = np.array([0, 8, 16, 24], np.uint32)
    qlo = np.stack([(q[:, 4 + 2 * a, None] >> shifts) & 255 for a in range(3)], 1).astype(np.float64)
    qhi = np.stack([(q[:, 5 + 2 * a, None] >> shifts) & 255 for a in range(3)], 1).astype(np.float64)
    dlo = origin[:, :, None] + qlo * step[:, :, None]
    dhi = origin[:, :, None] + qhi * step[:, :, None]
    v3 = np.broadcast_to(valid[:, None, :], lo.shape)
    assert np.all(dlo[v3] <= lo[v3]) and np.all(dhi[v3] >= hi[v3])
    assert np.all(qlo[~v3] == 255) and np.all(qhi[~v3] == 0)
    ref32 = f[:, 24:28].view(np.int32)
    refq = q[:, 12:16].view(np.int32)
    assert np.array_equal(refq[valid], ref32[valid])
    assert np.all(refq[~valid] == np.iinfo(np.int32).min)
    # the grid is fine where the boxes are: a valid child's quantized box is at most 2 grid steps wider per side
    assert np.all((lo - dlo)[v3] <= 2 * np.broadcast_to(step[:, :, None], lo.shape)[v3])


def test_quantized_grid_range_is_checked(fresh_core):
    """A BVH4 node wider than the quantized grid reaches (255 * 2^27 per axis: box4q scales the ray's clamped
    reciprocal +-1e30 by 2^e, which must stay finite, lh2_box4.inc / k_quantize4) is refused with a scene error,
    not traversed with inf / NaN slabs."""
    from lighthouse2_amd.core import CoreError
    big = abi.tris_from_vertices(np.array([[-1e11, 0, 0], [0, 0, 5]], np.float32), np.array([[1e11, 0, 0], [1, 0, 5]], np.float32),
                                 np.array([[0, 1e11, 0], [0, 1, 5]], np.float32), 0)
    sc = scene.config2_scene(n=2000, width=64, height=36)
    sc.meshes.append(big)
    sc.instances.append((1, np.eye(4, dtype=np.float32)))
    sc.load_into(fresh_core)
    fresh_core.set_target(64, 36, 1)
    with pytest.raises(CoreError, match="quantized"):
        sc.render_frame(fresh_core)
        fresh_core.sync()


@pytest.mark.parametrize("gpu_tlas", [1, 0])
def test_stale_tlas_region_is_not_quantized(gpu_tlas):
    """The TLAS slots hold tlasCapacity nodes; a TLAS update writes only the nodes its tree has.  The rest is an earlier,
    larger TLAS or memory never written, which may hold huge finite boxes.  Round 4's range check (k_quantize4) fired on
    such memory (`test_traversal_variants_bitexact[7-1-2]`, fixed by NaN-filling the region at allocation, 651cce0);
    since round 5 the BVH4 copy and the quantizer touch only the TLAS's own nodes (rendercore.cpp UpdateToplevel).  Here
    both slots are filled with 3e38 (finite: it passes k_quantize4's validity test and needs a grid exponent far past
    LH2_QEXP_MAX) before an instance update: the frame must render, equal to the same frames without the fill."""
    from lighthouse2_amd.core import RenderCore

    def run(poison):
        c = RenderCore(device=0)
        try:
            c.setting("gpuTlas", gpu_tlas)
            sc = scene.instanced_scene(meshes=6, tris_per_mesh=2000, width=64, height=36, grid=3, spacing=12.0)
            sc.load_into(c)
            c.set_target(64, 36, 1)
            sc.render_frame(c, converge=1)
            c.sync()
            if poison:
                c.debug_poison_tlas(3e38)
            scene.animate_instances(sc, 1)
            for k, (mesh, T) in enumerate(sc.instances[:4]):   # fewer instances: a smaller TLAS than the slot held
                c.set_instance(k, mesh, T)
            c.set_instance(4, -1, None)
            c.update_toplevel()
            sc.render_frame(c, converge=0)
            c.sync()
            return c.accumulator(), c.ray_counts()
        finally:
            c.close()

    a, ca = run(False)
    b, cb = run(True)
    assert np.array_equal(ca, cb)
    assert np.any(a[..., :3] != 0)
    assert rel_l2(b[..., :3], a[..., :3]) <= 1e-6
    assert np.array_equal(a[..., 3], b[..., 3])
