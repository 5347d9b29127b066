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


def test_gather_ordering_under_a_lagging_device0():
    """The gather of frame f must read frame f's rows even when the host has queued frame f + 1 and
    the ranks > 0 have rendered and packed it before device 0 copies frame f (multidevice.cpp: the send
    buffers are double-buffered by frame parity, and a pack waits for device 0's copy out of its buffer
    two frames back).  Device 0 idles 30 ms before every gather (setting "gatherStallUs"); four
    converging frames are queued back to back with no host synchronisation, each finalized frame copied
    on the core stream into its own device buffer (the headless display copy); every one of them must
    equal the single-device core's frame."""
    import torch
    w, h, frames = 160, 96, 4
    sc = scene.room_scene(30000, w, h)
    st = (("maxPathLength", 4),)
    ref = []
    c = RenderCore(device=0)
    try:
        for k, v in st:
            c.setting(k, v)
        sc.load_into(c)
        c.set_target(w, h, 1)
        for f in range(frames):
            sc.render_frame(c, converge=1 if f == 0 else 0)
            ref.append(c.frame())
    finally:
        c.close()
    c = RenderCore(device=0)
    try:
        c.setting("deviceCount", 3)
        c.setting("gatherStallUs", 30000)
        for k, v in st:
            c.setting(k, v)
        sc.load_into(c)
        c.set_target(w, h, 1)
        bufs = [torch.zeros((h, w, 4), dtype=torch.float32, device="cuda") for _ in range(frames)]
        torch.cuda.synchronize()
        for f in range(frames):
            sc.render_frame(c, converge=1 if f == 0 else 0)
            c.copy_frame_async(bufs[f].data_ptr())
        c.sync()
        got = [b.cpu().numpy() for b in bufs]
    finally:
        c.close()
    for f in range(frames):
        r = rel_l2(got[f][..., :3], ref[f][..., :3])
        print(f"frame {f}: rel-L2 vs one device {r:.2e}")
        assert r <= 1e-6, (f, r)


def test_repeated_settings_each_frame():
    """RenderSystem::Render sends six settings before every Render (rendersystem.cpp:231-236): with
    several devices, repeated values are applied once, and a changed value still reaches every sub-core."""
    w, h = 64, 40
    sc = scene.config2_scene(n=3000, width=w, height=h, sky=True)
    c = RenderCore(device=0)
    try:
        c.setting("deviceCount", 2)
        sc.load_into(c)
        c.set_target(w, h, 1)
        for f in range(3):
            for name, v in (("epsilon", 1e-4), ("clampValue", 10.0), ("clampDirect", 1.0), ("clampIndirect", 1.0),
                            ("filter", 0.0), ("TAA", 0.0)):
                c.setting(name, v)
            sc.render_frame(c, converge=1 if f == 0 else 0)
        a3 = c.accumulator()
        sc.render_frame(c, converge=1, clamp=0.05)   # changed: every sub-core clamps harder
        a_low = c.accumulator()
    finally:
        c.close()
    ref = RenderCore(device=0)
    try:
        sc.load_into(ref)
        ref.set_target(w, h, 1)
        sc.render_frame(ref, converge=1, clamp=0.05)
        b_low = ref.accumulator()
    finally:
        ref.close()
    assert np.isfinite(a3).all() and a3[..., :3].max() > a_low[..., :3].max()
    assert rel_l2(a_low[..., :3], b_low[..., :3]) <= 1e-6


@pytest.mark.parametrize("devices", [2, 3])
def test_blas_built_once_per_mesh(devices):
    """the in-core multi-device path builds each mesh's BLAS once on the host and uploads it to every
    sub-core (RenderCore::AdoptGeometry shares core 0's deferred build), instead of one build per device.  The process's
    CPU build count ("blasBuilds") grows by the mesh count whatever deviceCount is, and the frame still equals the
    one-device frame."""
    w, h = 96, 54
    sc = scene.instanced_scene(meshes=4, tris_per_mesh=3000, width=w, height=h, grid=2, spacing=12.0)

    def builds_during(n):
        c = RenderCore(device=0)
        try:
            b0 = c.get_setting("blasBuilds")
            if n > 1:
                c.setting("deviceCount", n)
            sc.load_into(c)
            c.set_target(w, h, 1)
            sc.render_frame(c, converge=1)
            return c.get_setting("blasBuilds") - b0, c.accumulator()
        finally:
            c.close()

    b1, a1 = builds_during(1)
    bn, an = builds_during(devices)
    assert b1 == len(sc.meshes) and bn == len(sc.meshes), (b1, bn)
    assert rel_l2(an[..., :3], a1[..., :3]) <= 1e-6
