"""GPU parity at the BASELINE workload sizes (configs 2, 3 and 5 of BASELINE.json).

The miniature parity tests (test_gpu_parity.py) cover every code path on small scenes; these run the
benchmarked configurations themselves through the C-ABI against the CPU oracle, so deep trees
(config 2: BVH depth 31, config 3: depth 46), LDS-stack spills at real depth, full-size ray / shadow
buffers, 100 instanced BLAS with a per-frame TLAS rebuild and the 24-bit path-index packing at
16,588,800 paths (config 5, `kernels/camera.h:92`) are exercised at the sizes the bench times.

Bar: identical per-bounce ray counts, accumulator relative L2 <= 1e-4 (north_star), bit-exact hit
records {t, triid, instid, uv16}; and the HIP traversal against the reference's own traversal
(RenderCore_Bart BVH2::Traverse, compiled from /root/reference into the committed golden sample
tests/golden/bart_config2_sample.npz) with the thresholds test_golden.py applies to the oracle.
"""
import pathlib

import numpy as np
import pytest

from lighthouse2_amd import abi, scene
from oracle.oracle import Oracle

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

REL_L2_TOL = 1e-4
GOLD = pathlib.Path(__file__).resolve().parent / "golden"


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _pair(sc, w, h, spp=1, settings=()):
    from lighthouse2_amd.core import RenderCore
    core = RenderCore(device=0)
    o = Oracle()
    for tgt in (core, o):
        sc.load_into(tgt)
        tgt.set_target(w, h, spp)
        for k, v in settings:
            tgt.setting(k, v)
    return core, o


def _frame_parity(core, o, sc, what):
    sc.render_frame(core)
    sc.render_frame(o)
    cg, co = core.ray_counts(), o.ray_counts()
    assert np.array_equal(cg, co), (what, cg, co)
    ag, ao = core.accumulator(), o.accumulator()
    r = rel_l2(ag[..., :3], ao[..., :3])
    print(f"{what}: rays {co[:4].tolist()} shadow {int(co[16])} rel-L2 {r:.2e}")
    assert r <= REL_L2_TOL, (what, r)
    assert rel_l2(ag[..., 3], ao[..., 3]) <= 1e-6
    st = core.stats()
    assert st.primaryRayCount == co[0] and st.bounce1RayCount == co[1]
    return co


@pytest.fixture(scope="module")
def config2():
    """Config 2 at its bench size: 100k xorshift triangles, 1920x1080, 1 spp."""
    sc = scene.config2_scene(n=100_000)
    core, o = _pair(sc, 1920, 1080)
    yield sc, core, o
    core.close()
    o.close()


@pytest.mark.timeout(300)
def test_config2_fullsize_frame(config2):
    sc, core, o = config2
    info = core.scene_info()
    assert info["tris"] == 100_000 and info["max_depth"] >= 25
    co = _frame_parity(core, o, sc, "config2 1920x1080")
    assert co[0] == 1920 * 1080 and co[1] > 1_900_000


@pytest.mark.timeout(300)
def test_config2_fullsize_primary_and_bounce_hits_bitexact(config2):
    """Every one of the frame's 2,073,600 primary rays and the diffuse bounce rays they spawn: the
    HIP hit records equal the oracle's bit for bit."""
    sc, core, o = config2
    for tgt in (core, o):
        tgt.setting("epsilon", 1e-4)
    O4, D4, _ = o.generate_eye_rays(sc.view, 0, 0)
    hg = core.trace_closest(O4, D4)
    ho = o.trace_closest(O4, D4)
    assert np.array_equal(hg, ho), np.argwhere((hg != ho).any(1))[:10]
    bo, bd = scene.bounce_rays(sc.meshes[0], O4, D4, ho)
    assert len(bo) > 1_900_000
    hg = core.trace_closest(bo, bd)
    hb = o.trace_closest(bo, bd)
    assert np.array_equal(hg, hb), np.argwhere((hg != hb).any(1))[:10]


def test_config2_hip_traversal_matches_reference_sample(config2):
    """The HIP closest hit against RenderCore_Bart BVH2::Traverse (bvh.cpp:258-302, common.h:19-50),
    compiled from the reference sources: the 64x36 golden sample of config-2 primary rays.  Same
    thresholds as the oracle's pin (test_golden.py): Bart renormalises the direction and computes 1/a
    in double, so t agrees to a few ulp; hit/miss and the face normal agree."""
    sc, core, o = config2
    g = np.load(GOLD / "bart_config2_sample.npz")
    n = len(g["org"])
    assert n >= 2304
    O4 = np.concatenate([g["org"], np.full((n, 1), 1e-4, np.float32)], 1)
    D4 = np.concatenate([g["dir"], np.full((n, 1), 1e34, np.float32)], 1)
    hits = core.trace_closest(O4, D4)
    ghit = hits[:, 1] != 0xFFFFFFFF
    bhit = g["t"] < 1e30
    assert (ghit == bhit).mean() >= 0.999
    both = ghit & bhit
    assert both.sum() > 0.5 * n
    t_g = hits[both, 0].view(np.float32)
    t_b = g["t"][both]
    assert np.max(np.abs(t_g - t_b) / t_b) < 1e-5
    tris = sc.meshes[0]
    tri = hits[both, 1].astype(np.int64)
    N = np.stack([tris[tri, abi.TRI["Nx"]], tris[tri, abi.TRI["Ny"]], tris[tri, abi.TRI["Nz"]]], 1)
    assert np.mean(np.all(np.abs(N - g["normal"][both]) < 1e-6, axis=1)) >= 0.999


@pytest.mark.timeout(400)
def test_config3_fullsize_frame():
    """Config 3 at its bench size: the 1M-triangle procedural room (specular chains, glass, smooth
    spheres, two area lights: NEE, shadow rays, MIS), 1920x1080, 1 spp, maxPathLength 4."""
    sc = scene.room_scene(1_000_000)
    core, o = _pair(sc, 1920, 1080, settings=(("maxPathLength", 4),))
    try:
        info = core.scene_info()
        assert info["tris"] >= 999_000 and info["max_depth"] >= 40
        co = _frame_parity(core, o, sc, "config3 room 1M 1920x1080")
        assert co[3] > 0 and co[4] == 0 and co[16] > 2_000_000
        # a second, converging frame: the accumulator sums both samples
        sc.render_frame(core, converge=0)
        sc.render_frame(o, converge=0)
        assert np.array_equal(core.ray_counts(), o.ray_counts())
        assert rel_l2(core.frame()[..., :3], o.frame()[..., :3]) <= REL_L2_TOL
    finally:
        core.close()
        o.close()


@pytest.mark.timeout(600)
def test_config5_fullsize_instanced_8spp():
    """Config 5 at its bench size: 100 distinct 100k-triangle meshes (10M triangles), each placed by
    one instance, a per-frame instance update (SetInstance x 100 + UpdateToplevel: TLAS rebuilt on the
    device), 1920x1080 at 8 spp = 16,588,800 paths, just under the 24-bit path-index cap."""
    w, h, spp = 1920, 1080, 8
    assert w * h * spp == 16_588_800 < (1 << 24)
    sc = scene.instanced_scene(meshes=100, tris_per_mesh=100_000, width=w, height=h)
    core, o = _pair(sc, w, h, spp)
    try:
        assert core.scene_info()["instances"] == 100
        scene.animate_instances(sc, 1)
        for tgt in (core, o):
            for k, (mesh, T) in enumerate(sc.instances):
                tgt.set_instance(k, mesh, T)
            tgt.update_toplevel()
        # hit records through the rotated instances, bit-exact: 131072 rays aimed into the field
        rng = np.random.default_rng(11)
        n = 131072
        org = np.stack([rng.uniform(-70, 70, n), rng.uniform(20, 60, n), rng.uniform(-90, -60, n)], 1).astype(np.float32)
        tgt_pts = np.stack([rng.uniform(-60, 60, n), rng.uniform(-5, 5, n), rng.uniform(-60, 60, n)], 1)
        d = (tgt_pts - org).astype(np.float32)
        d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
        O4 = np.concatenate([org, np.full((n, 1), 1e-4, np.float32)], 1)
        D4 = np.concatenate([d, np.full((n, 1), 1e34, np.float32)], 1)
        hg, ho = core.trace_closest(O4, D4), o.trace_closest(O4, D4)
        assert (ho[:, 1] != 0xFFFFFFFF).mean() > 0.3
        assert len(np.unique(ho[ho[:, 1] != 0xFFFFFFFF, 2])) >= 50      # hits spread over many instances
        assert np.array_equal(hg, ho), np.argwhere((hg != ho).any(1))[:10]
        co = _frame_parity(core, o, sc, "config5 100x100k 1920x1080 8spp")
        assert co[0] == 16_588_800
    finally:
        core.close()
        o.close()


@pytest.mark.timeout(900)
def test_config4_fullsize_partitioned_frame():
    """Config 4 at its size: the config-3 room (1M triangles, maxPathLength 4, lights) at 3840x2160,
    1 spp = 8,294,400 paths, the frame split over 8 sub-cores in 8-row bands (setting "deviceCount" 8:
    the partition, the per-rank 4K accumulators and frame buffers, the 2N shadow buffers, the row-map
    finalize and the gather of multidevice.cpp; on a one-GPU box the 8 sub-cores share device 0).
    Against the single-device core: identical per-bounce ray counts, accumulator within 1e-6.  Against
    the oracle: rank 0's bands (set_tile_bands(0, 8, 8), the pixels of pathtracer.h:79-80 it owns)
    within 1e-4.  Reference sizing: RenderCore_OptixPrime_B/rendercore.cpp:149-209."""
    from lighthouse2_amd.core import RenderCore
    W, H, N, BAND = 3840, 2160, 8, 8
    sc = scene.room_scene(1_000_000, W, H)
    st = (("maxPathLength", 4),)

    def render(devices):
        c = RenderCore(device=0)
        try:
            if devices > 1:
                c.setting("deviceCount", devices)
            for k, v in st:
                c.setting(k, v)
            sc.load_into(c)
            c.set_target(W, H, 1)
            sc.render_frame(c)
            return c.accumulator(), c.ray_counts(), c.stats()
        finally:
            c.close()

    a8, c8, s8 = render(N)
    a1, c1, s1 = render(1)
    assert c1[0] == W * H and c1[16] > 8_000_000
    assert np.array_equal(c8, c1), (c8, c1)
    r = rel_l2(a8[..., :3], a1[..., :3])
    print(f"config4 4K: rays {c1[:4].tolist()} shadow {int(c1[16])}; 8 sub-cores vs 1: rel-L2 {r:.2e}")
    assert r <= 1e-6
    assert np.array_equal(a8[..., 3], a1[..., 3])
    assert (s8.primaryRayCount, s8.bounce1RayCount, s8.totalShadowRays) == (s1.primaryRayCount, s1.bounce1RayCount, s1.totalShadowRays)
    o = Oracle()
    try:
        sc.load_into(o)
        for k, v in st:
            o.setting(k, v)
        o.set_target(W, H, 1)
        o.set_tile_bands(0, N, BAND)
        sc.render_frame(o)
        ao = o.accumulator()
    finally:
        o.close()
    rows = np.concatenate([np.arange(y, min(y + BAND, H)) for y in range(0, H, N * BAND)])
    r0 = rel_l2(a8[rows, :, :3], ao[rows, :, :3])
    print(f"config4 4K rank 0 bands ({len(rows)} rows) vs oracle: rel-L2 {r0:.2e}")
    assert r0 <= REL_L2_TOL
    assert rel_l2(a8[rows, :, 3], ao[rows, :, 3]) <= 1e-6
