"""In-process multi-device mode of the core (setting "deviceCount", csrc/multidevice.cpp).

One RenderSystem process loads one core (lib/RenderSystem/core_api_base.cpp:97-132); with
deviceCount N the core itself deals the frame's 8-row bands round-robin over N sub-cores (one per
HIP device), renders them concurrently and gathers the accumulator rows to device 0 by peer copy.
On a one-GPU box the sub-cores share device 0, which runs the same partition, unpack and finalize
with local copies: the gathered frame must equal the single-device frame (SURVEY.md §8e,
"partition invariance").  Multi-GPU placement itself is covered by the driver's 8-GPU runs.
"""
import numpy as np
import pytest

from lighthouse2_amd import scene
from lighthouse2_amd.core import CoreError, RenderCore

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _render(sc, w, h, devices, frames=2, spp=1, settings=()):
    c = RenderCore(device=0)
    try:
        if devices > 1:
            c.setting("deviceCount", devices)
        for k, v in settings:
            c.setting(k, v)
        sc.load_into(c)
        c.set_target(w, h, spp)
        c.set_probe(w // 3, h // 2)
        for f in range(frames):
            sc.render_frame(c, converge=1 if f == 0 else 0)
        return c.accumulator(), c.frame(), c.ray_counts(), c.stats()
    finally:
        c.close()


@pytest.mark.parametrize("devices", [2, 3])
def test_device_partition_equals_single_device(devices):
    """Lit room, depth 4, two converging frames at 2 spp: accumulator, finalized frame, per-bounce ray
    counts and CoreStats of the N-sub-core core equal the one-device core's."""
    w, h = 160, 90                    # 90 rows: the last band is partial
    sc = scene.room_scene(30000, w, h)
    st = (("maxPathLength", 4),)
    a1, f1, c1, s1 = _render(sc, w, h, 1, spp=2, settings=st)
    an, fn, cn, sn = _render(sc, w, h, devices, spp=2, settings=st)
    assert np.array_equal(c1, cn), (c1, cn)
    assert rel_l2(an[..., :3], a1[..., :3]) <= 1e-6
    assert np.array_equal(an[..., 3], a1[..., 3])
    assert rel_l2(fn[..., :3], f1[..., :3]) <= 1e-6
    assert (sn.primaryRayCount, sn.bounce1RayCount, sn.totalShadowRays) == (s1.primaryRayCount, s1.bounce1RayCount, s1.totalShadowRays)
    assert (sn.probedTriid, sn.probedInstid) == (s1.probedTriid, s1.probedInstid)


def test_device_partition_config2_frame():
    """The bench's config-2 frame (no lights: terminal shading, single-instance start) split over 2."""
    w, h = 320, 180
    sc = scene.config2_scene(n=20000, width=w, height=h, sky=True)
    a1, _, c1, _ = _render(sc, w, h, 1, frames=1)
    a2, _, c2, _ = _render(sc, w, h, 2, frames=1)
    assert np.array_equal(c1, c2)
    assert rel_l2(a2[..., :3], a1[..., :3]) <= 1e-6


def test_device_count_after_scene_is_an_error():
    w, h = 64, 36
    sc = scene.config2_scene(n=2000, width=w, height=h)
    c = RenderCore(device=0)
    try:
        sc.load_into(c)
        c.set_target(w, h, 1)
        with pytest.raises(CoreError, match="deviceCount"):
            c.setting("deviceCount", 2)
        c.setting("deviceCount", 1)          # unchanged: no error
        sc.render_frame(c)
        with pytest.raises(CoreError, match="deviceCount"):
            c.setting("deviceCount", 4)
    finally:
        c.close()


def test_partition_extensions_refused_with_several_devices():
    c = RenderCore(device=0)
    try:
        c.setting("deviceCount", 2)
        with pytest.raises(CoreError, match="deviceCount"):
            c.set_tile_bands(0, 2, 8)
    finally:
        c.close()
