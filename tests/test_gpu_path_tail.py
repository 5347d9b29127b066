"""GPU parity of the path tail (setting pathTail, k_trace_path4d): the bounces from pathTail on are
traced and shaded in one launch, each lane shading its finished closest-hit queries with k_shade's code
and walking on with the extension ray.  Against the CPU oracle (pathtracer.h:54-245, one launch pair
per bounce in the reference): identical per-bounce ray counts (rayCount log, counted by the launch's
per-length atomics), accumulator rel-L2 <= 1e-4, and the same frame with the tail off to float
summation order."""
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


def _scene(kind, w, h):
    if kind == "room":                    # lit: NEE shadow rays from every vertex, glass and mirrors
        return scene.room_scene(40000, w, h)
    if kind == "specular":                # no lights: k_trace_path4d<true>, long specular chains
        sc = scene.config2_scene(n=20000, width=w, height=h, sky=True)
        sc.area_lights = []
        sc.materials.append(abi.make_material((0.9, 0.9, 0.9), roughness=0.0))
        sc.meshes[0].view(np.uint32)[::2, abi.TRI["material"]] = 1
        return sc
    sc = scene.instanced_scene(meshes=4, tris_per_mesh=4000, width=w, height=h, grid=2, spacing=10.0)
    scene.animate_instances(sc, 1)        # several instances: rays re-enter their instance after a shade batch
    sc.sky = scene.gradient_sky(64, 32)
    return sc


@pytest.mark.parametrize("kind,depth", [("room", 4), ("room", 6), ("specular", 5), ("instanced", 4)])
@pytest.mark.parametrize("tail", [2, 3])
@pytest.mark.parametrize("waves", [0, 4])
def test_path_tail_frame_parity(fresh_core, kind, depth, tail, waves):
    """The path tail against the oracle and against a launch pair per bounce; waves 4: the kernel variant compiled for
    4 waves per SIMD (128 VGPRs, spills), which large frames use (pathTailWaves; 0: by frame size, 3 here)."""
    w, h = 128, 72
    sc = _scene(kind, w, h)
    o = _load_both(fresh_core, sc, w, h)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", depth)
    fresh_core.setting("pathTail", tail)
    fresh_core.setting("pathTailWaves", waves)
    for f in range(2):
        sc.render_frame(fresh_core, converge=1 if f == 0 else 0)
        sc.render_frame(o, converge=1 if f == 0 else 0)
        cg, co = fresh_core.ray_counts(), o.ray_counts()
        assert np.array_equal(cg, co), (f, cg[:8], co[:8])
    assert co[1] > 0 and (kind == "instanced" or co[tail - 1] > 0), co[:8]
    ag, ao = fresh_core.accumulator(), o.accumulator()
    assert rel_l2(ag[..., :3], ao[..., :3]) <= REL_L2_TOL
    assert rel_l2(ag[..., 3], ao[..., 3]) <= 1e-6
    st = fresh_core.stats()
    assert st.totalExtensionRays == int(co[:16].sum())
    # the same two frames with a launch pair per bounce
    fresh_core.setting("pathTail", 0)
    for f in range(2):
        sc.render_frame(fresh_core, converge=1 if f == 0 else 0)
    a0 = fresh_core.accumulator()
    assert rel_l2(ag[..., :3], a0[..., :3]) <= 1e-6


@pytest.mark.parametrize("batch", [1, 7, 64])
def test_path_tail_shade_batches(fresh_core, batch):
    """Every shade batch size (1: shade as soon as a query finishes; 64: only when no lane walks)."""
    w, h = 96, 54
    sc = _scene("room", w, h)
    o = _load_both(fresh_core, sc, w, h)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", 5)
    fresh_core.setting("pathTail", 2)
    fresh_core.setting("pathTailBatch", batch)
    sc.render_frame(fresh_core)
    sc.render_frame(o)
    assert np.array_equal(fresh_core.ray_counts(), o.ray_counts())
    assert rel_l2(fresh_core.accumulator()[..., :3], o.accumulator()[..., :3]) <= REL_L2_TOL


def test_path_tail_spp_and_pass_past_256(fresh_core):
    """Several samples per pixel (path index -> sample) and passes past the blue-noise range (random
    numbers from the per-path seed, R0 of the lane's own path length)."""
    w, h = 32, 18
    sc = _scene("room", w, h)
    o = _load_both(fresh_core, sc, w, h, spp=4)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", 4)
    fresh_core.setting("pathTail", 3)
    for f in range(66):      # 66 x 4 = 264 samples: the last frames run past sample 256
        sc.render_frame(fresh_core, converge=1 if f == 0 else 0)
        sc.render_frame(o, converge=1 if f == 0 else 0)
        if f in (0, 65):
            assert np.array_equal(fresh_core.ray_counts(), o.ray_counts())
    assert rel_l2(fresh_core.accumulator()[..., :3], o.accumulator()[..., :3]) <= REL_L2_TOL


@pytest.mark.parametrize("factor", [0.5, 2.0])
def test_heavy_first_packets_frames(fresh_core, factor):
    """Heavy-first primary packets (setting packetHeavy): from the second frame on, the packets that took
    more than factor x the previous frame's mean node steps are taken first and skipped in the in-order
    pass.  Every packet is traced exactly once: frame after frame the ray counts and the accumulator
    match the oracle; a new target size (a new packet layout) starts over."""
    w, h = 160, 96
    sc = scene.config2_scene(n=20000, width=w, height=h, sky=True)
    o = _load_both(fresh_core, sc, w, h)
    fresh_core.setting("packetHeavy", factor)
    assert fresh_core.get_setting("usePackets") == 1
    for f in range(4):
        sc.render_frame(fresh_core, converge=1 if f == 0 else 0)
        sc.render_frame(o, converge=1 if f == 0 else 0)
        assert np.array_equal(fresh_core.ray_counts(), o.ray_counts()), f
    assert rel_l2(fresh_core.accumulator()[..., :3], o.accumulator()[..., :3]) <= REL_L2_TOL
    w2, h2 = 96, 64
    sc2 = scene.config2_scene(n=20000, width=w2, height=h2, sky=True)
    fresh_core.set_target(w2, h2, 1)
    o2 = Oracle()
    sc2.load_into(o2)
    o2.set_target(w2, h2, 1)
    for f in range(3):
        sc2.render_frame(fresh_core, converge=1 if f == 0 else 0)
        sc2.render_frame(o2, converge=1 if f == 0 else 0)
        assert np.array_equal(fresh_core.ray_counts(), o2.ray_counts()), f
    assert rel_l2(fresh_core.accumulator()[..., :3], o2.accumulator()[..., :3]) <= REL_L2_TOL


@pytest.mark.parametrize("blocks,tail,side,final", [(0, 2, 0, 6), (3, 2, 0, 6), (0, 3, 0, 6), (3, 3, 0, 0), (0, 3, 7, 6),
                                                    (0, 4, 2, 3)])
def test_shadow_overlap(fresh_core, blocks, tail, side, final):
    """shadowOverlap: the shadow rays queued before the path tail are traced on the side stream beside it
    (their segment counts snapshotted by the shade launch before the tail; the path tail at 2 or 3 blocks per CU
    by frame size, or pathTailBlocks; the side launch at sideBlocks per CU, 0: the trace grid's), and the final shadow
    launch (finalShadowBlocks per CU, 4 by default, 0: the trace grid's) starts behind them.
    Every shadow ray is traced once: the same ray counts and occlusion as the oracle, three converging frames within
    rel-L2 1e-4 of it, and within float summation order of the frames traced with the overlap off."""
    w, h = 128, 72
    sc = _scene("room", w, h)
    o = _load_both(fresh_core, sc, w, h)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", 4)
    fresh_core.setting("pathTail", tail)
    fresh_core.setting("pathTailBlocks", blocks)
    fresh_core.setting("sideBlocks", side)
    fresh_core.setting("finalShadowBlocks", final)
    res = {}
    for ov in (1, 0):
        fresh_core.setting("shadowOverlap", ov)
        for f in range(3):
            sc.render_frame(fresh_core, converge=1 if f == 0 else 0)
            if ov:
                sc.render_frame(o, converge=1 if f == 0 else 0)
                assert np.array_equal(fresh_core.ray_counts(), o.ray_counts()), f
        res[ov] = (fresh_core.accumulator(), fresh_core.stats())
    ag, st = res[1]
    co = o.ray_counts()
    assert co[16] > 0 and st.totalShadowRays == co[16], (st.totalShadowRays, co[16])
    assert rel_l2(ag[..., :3], o.accumulator()[..., :3]) <= REL_L2_TOL
    assert rel_l2(ag[..., :3], res[0][0][..., :3]) <= 1e-6


@pytest.mark.parametrize("blocks", [1, 8, 40, 64])
def test_shade_grid(fresh_core, blocks):
    """The shade launches' grid (shadeBlocks per CU; 0, the default: about 1.3 paths per thread, between the trace grid
    and 24 blocks per CU, RenderCore::kShadePathsPerThread / kShadeMaxBlocks): each block walks its segment with a static
    stride, so every grid must shade every path once; the same ray counts as the oracle and the frame within float
    summation order of the default grid's."""
    w, h = 128, 72
    sc = _scene("room", w, h)
    o = _load_both(fresh_core, sc, w, h)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", 4)
    res = []
    for b in (0, blocks):
        fresh_core.setting("shadeBlocks", b)
        for f in range(2):
            sc.render_frame(fresh_core, converge=1 if f == 0 else 0)
            if not res:
                sc.render_frame(o, converge=1 if f == 0 else 0)
        res.append((fresh_core.accumulator(), fresh_core.ray_counts()))
    assert np.array_equal(res[1][1], o.ray_counts())
    assert rel_l2(res[1][0][..., :3], o.accumulator()[..., :3]) <= REL_L2_TOL
    assert rel_l2(res[1][0][..., :3], res[0][0][..., :3]) <= 1e-6
