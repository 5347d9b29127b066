"""GPU parity of the shadow backfill (setting shadowBackfill, k_trace_closest4d_bf): once a closest-hit
launch's own queues are dry, its idle lanes trace shadow rays queued by earlier bounces (any hit + the
fused finalizeConnection of connections.h:22-44), claimed from the final shadow launch's work-queue heads
so that launch traces exactly the rest.  Against the CPU oracle (the reference traces every shadow ray in
one launch after the bounce loop, rendercore.cpp:575-592): identical per-bounce and shadow ray counts,
accumulator rel-L2 <= 1e-4, and the same frames with the backfill off to float summation order (every
shadow ray adds its potential exactly once).  Off by default: the backfilled shadow rays slow the closest-hit
rays still in flight, which set the launch's end (profiles/r02zg_ab_shadow_backfill.txt)."""
import numpy as np
import pytest

from lighthouse2_amd import scene
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

REL_L2_TOL = 1e-4


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _scene(kind, w, h):
    if kind == "room":            # one instance: rays start inside it
        return scene.room_scene(40000, w, h)
    # two instances (random triangles + the light quad): shadow lanes leave a BLAS and reload their ray
    return scene.config2_scene(n=20000, width=w, height=h, sky=True, light=True)


@pytest.mark.parametrize("kind,depth,tail", [("room", 4, 3), ("room", 4, 0), ("room", 6, 0), ("twoinst", 4, 0),
                                             ("twoinst", 5, 3)])
def test_shadow_backfill_frame_parity(fresh_core, kind, depth, tail):
    w, h = 128, 72
    sc = _scene(kind, w, h)
    sc.load_into(fresh_core)
    fresh_core.set_target(w, h, 1)
    o = Oracle()
    sc.load_into(o)
    o.set_target(w, h, 1)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", depth)
    fresh_core.setting("pathTail", tail)
    fresh_core.setting("shadowBackfill", 1)
    assert fresh_core.get_setting("shadowBackfill") == 1
    for f in range(2):
        sc.render_frame(fresh_core, converge=1 if f == 0 else 0)
        sc.render_frame(o, converge=1 if f == 0 else 0)
        cg, co = fresh_core.ray_counts(), o.ray_counts()
        assert np.array_equal(cg, co), (f, cg[:8], cg[16], co[:8], co[16])
    assert co[16] > 0 and co[1] > 0
    ag, ao = fresh_core.accumulator(), o.accumulator()
    assert rel_l2(ag[..., :3], ao[..., :3]) <= REL_L2_TOL
    # the same two frames without the backfill: every shadow ray in the final launch
    fresh_core.setting("shadowBackfill", 0)
    for f in range(2):
        sc.render_frame(fresh_core, converge=1 if f == 0 else 0)
    assert np.array_equal(fresh_core.ray_counts(), co)
    a0 = fresh_core.accumulator()
    assert rel_l2(ag[..., :3], a0[..., :3]) <= 1e-6


@pytest.mark.parametrize("refill", [1, 64])
def test_shadow_backfill_refill_extremes(fresh_core, refill):
    """Claims of one ray (refill 1: a claim as soon as a lane is idle) and of whole waves (64)."""
    w, h = 96, 54
    sc = _scene("room", w, h)
    sc.load_into(fresh_core)
    fresh_core.set_target(w, h, 1)
    fresh_core.setting("maxPathLength", 5)
    fresh_core.setting("pathTail", 0)
    fresh_core.setting("refill", refill)
    fresh_core.setting("shadowBackfill", 1)
    sc.render_frame(fresh_core)
    a1, c1 = fresh_core.accumulator(), fresh_core.ray_counts()
    fresh_core.setting("shadowBackfill", 0)
    sc.render_frame(fresh_core)
    assert np.array_equal(fresh_core.ray_counts(), c1)
    assert rel_l2(a1[..., :3], fresh_core.accumulator()[..., :3]) <= 1e-6
