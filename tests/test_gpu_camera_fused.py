"""GPU parity of the camera fused into the primary packet launch (setting cameraFused, k_trace_primary_packet):
the packet launch makes each path's primary ray itself (camera.h:39-111, the code of k_camera) and does the
camera launch's frame resets, its work-queue heads alternating between two slots from frame to frame, and the
heavy-packet block the next frame records into zeroed by the first shade launch.  Against the CPU oracle
(pathtracer.h:54-245 after generateEyeRays): identical per-bounce ray counts every frame, accumulator rel-L2
<= 1e-4, and the same frames with the camera launch (cameraFused 0) to float summation order; a restart in
the middle of the sequence exercises the accumulator reset of each pixel's first sample."""
import numpy as np
import pytest

from lighthouse2_amd import scene
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

REL_L2_TOL = 1e-4


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


# restart, converge, converge, restart, converge, converge: both head slots, each twice, and two restarts
SEQUENCE = (1, 0, 0, 1, 0, 0)


@pytest.mark.parametrize("kind", ["room", "config2"])
def test_camera_fused_frames(fresh_core, kind):
    w, h = 128, 72
    if kind == "room":
        sc = scene.room_scene(40000, w, h)
        depth = 4
    else:
        sc = scene.config2_scene(n=20000, width=w, height=h)
        depth = 2
    sc.load_into(fresh_core)
    fresh_core.set_target(w, h, 1)
    o = Oracle()
    sc.load_into(o)
    o.set_target(w, h, 1)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", depth)
    assert fresh_core.get_setting("cameraFused") == 1
    res = {}
    for fused in (1, 0):
        fresh_core.setting("cameraFused", fused)
        for f, conv in enumerate(SEQUENCE):
            sc.render_frame(fresh_core, converge=conv)
            if fused:
                sc.render_frame(o, converge=conv)
                assert np.array_equal(fresh_core.ray_counts(), o.ray_counts()), (f, fresh_core.ray_counts()[:6], o.ray_counts()[:6])
        res[fused] = fresh_core.accumulator()
    assert rel_l2(res[1][..., :3], o.accumulator()[..., :3]) <= REL_L2_TOL
    assert rel_l2(res[1][..., :3], res[0][..., :3]) <= 1e-6
    # the primary hit distances (the accumulator's w: first-vertex distance sum) are order-free sums of identical values
    assert np.array_equal(res[1][..., 3], res[0][..., 3])
