"""GPU parity of the camera fused into the primary packet launch (setting cameraFused, k_trace_primary_packet) and
of the frame overlap (setting frameOverlap).  The packet launch makes each path's primary ray itself (camera.h:39-111,
the code of k_camera) into primary buffers of its own, and runs on the core's ahead stream: beside the previous
frame's later bounces once that frame's shade launch before its path tail (or its first) is done, or behind the whole
previous frame after a restart or a scene change.  Consecutive frames use counters, work-queue heads and shadow streams of
their own parity; the frame's resets are a k_init_counters launch before the primary launch on the ahead stream; the
heavy-packet block the next frame records into is zeroed by the first shade launch (or, before a frame whose primary
launch may run ahead, by a memset on the ahead stream).  With earlyShade (default) the first shade launch of a frame after
one with a path tail follows its primary launch on the ahead stream too, beside the previous frame's path tail and shadow
launches.

Against the CPU oracle (pathtracer.h:54-245 after generateEyeRays): identical per-bounce ray counts every frame,
accumulator rel-L2 <= 1e-4; and frames queued back to back (no host synchronisation between them, so the primary
launches overlap the previous frames' tails) equal, to float summation order, the same frames without the overlap
and without the fusion.  Restarts in the sequence exercise the accumulator reset of each pixel's first sample."""
import numpy as np
import pytest

from lighthouse2_amd import scene
from lighthouse2_amd.core import RenderCore
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

REL_L2_TOL = 1e-4


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


# restart, converge x2, restart, converge x3: both head slots, each several times, and two restarts
SEQUENCE = (1, 0, 0, 1, 0, 0, 0)


def _scene(kind, w, h):
    if kind == "room":
        return scene.room_scene(40000, w, h), 4
    if kind == "instanced":
        sc = scene.instanced_scene(meshes=4, tris_per_mesh=4000, width=w, height=h, grid=2, spacing=10.0)
        sc.sky = scene.gradient_sky(64, 32)
        return sc, 3
    return scene.config2_scene(n=20000, width=w, height=h), 2


def _animate(sc, tgt, f):
    scene.animate_instances(sc, f)
    for k, (mesh, T) in enumerate(sc.instances):
        tgt.set_instance(k, mesh, T)
    tgt.update_toplevel()


# packets -1: the core's choice (packets for these scenes: the fused camera + packet launch); 0: primary rays traced per ray
# (config 5's case: round 6 overlaps those frames too, a camera launch + per-ray primary launch on the ahead stream)
@pytest.mark.parametrize("packets", [-1, 0])
@pytest.mark.parametrize("kind", ["room", "config2", "instanced"])
def test_camera_fused_frames(fresh_core, kind, packets):
    w, h = 128, 72
    sc, depth = _scene(kind, w, h)
    anim = kind == "instanced"            # instances move every frame: each primary launch waits for the update
    fresh_core.setting("packetPrimary", packets)
    sc.load_into(fresh_core)
    fresh_core.set_target(w, h, 1)
    o = Oracle()
    sc.load_into(o)
    o.set_target(w, h, 1)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", depth)
    assert fresh_core.get_setting("cameraFused") == 1 and fresh_core.get_setting("frameOverlap") == 1
    assert fresh_core.get_setting("earlyShade") == 1
    # per-frame ray counts against the oracle (synchronised after every frame)
    for f, conv in enumerate(SEQUENCE):
        if anim:
            _animate(sc, fresh_core, f), _animate(sc, o, f)
        sc.render_frame(fresh_core, converge=conv)
        sc.render_frame(o, converge=conv)
        assert np.array_equal(fresh_core.ray_counts(), o.ray_counts()), (f, fresh_core.ray_counts()[:6], o.ray_counts()[:6])
    ref = o.accumulator()
    res = {}
    # (cameraFused, frameOverlap, earlyShade)
    variants = ((1, 1, 1), (1, 1, 0), (1, 2, 0), (1, 0, 0), (0, 0, 0))
    for fused, overlap, early in variants:
        fresh_core.setting("cameraFused", fused)
        fresh_core.setting("frameOverlap", overlap)
        fresh_core.setting("earlyShade", early)
        for f, conv in enumerate(SEQUENCE):   # queued back to back: no synchronisation between frames
            if anim:
                _animate(sc, fresh_core, f)
            sc.render_frame(fresh_core, converge=conv)
        res[(fused, overlap, early)] = fresh_core.accumulator()
        assert np.array_equal(fresh_core.ray_counts(), o.ray_counts()), (fused, overlap, early)
    a = res[variants[0]]
    assert rel_l2(a[..., :3], ref[..., :3]) <= REL_L2_TOL
    for k in variants[1:]:
        assert rel_l2(a[..., :3], res[k][..., :3]) <= 1e-6, k
        # the first-vertex distances (w): one addition per pixel per frame, in frame order: bit-identical
        assert np.array_equal(a[..., 3], res[k][..., 3]), k


@pytest.mark.parametrize("packets", [-1, 0])
@pytest.mark.parametrize("kind", ["room", "config2", "instanced"])
def test_animated_restart_frames(fresh_core, kind, packets):
    """tinyapp's animated loop (apps/tinyapp/main.cpp:98-118): SetInstance + UpdateToplevel and Render(Restart) every
    frame.  An instance-only UpdateToplevel writes the TLAS slot no frame in flight reads, on the ahead stream behind
    the last frame that read it, and a restart beside the previous frame zeroes the accumulator on the core stream, so
    these frames overlap too.  Every prefix of the sequence, queued back to back, equals the same frames serialised
    (frameOverlap 0): the same per-bounce ray counts, the accumulator to float summation order (w bit for bit).  A
    second UpdateToplevel before a frame (the slot the frame in flight reads) must wait for that frame."""
    w, h = 96, 64
    sc, depth = _scene(kind, w, h)
    if kind == "config2":
        sc.sky = scene.gradient_sky(64, 32)   # something to accumulate (config 2 has no lights)
    base = list(sc.instances)
    fresh_core.setting("packetPrimary", packets)
    sc.load_into(fresh_core)
    fresh_core.set_target(w, h, 1)
    fresh_core.setting("maxPathLength", depth)

    def turn(f):
        for k, (mesh, T) in enumerate(base):
            M = (scene.rotation_y(0.02 * (f + 1) * (1 + k % 3)) @ T).astype(np.float32) if kind != "instanced" else None
            if M is None:
                M = scene.rotation_y(0.3 * (f + 1) * (1 + k % 3))
                M[:3, 3] = T[:3, 3]
            fresh_core.set_instance(k, mesh, M)
        fresh_core.update_toplevel()

    def run(n, overlap, double):
        fresh_core.setting("frameOverlap", overlap)
        for f in range(n):
            turn(f)
            if double and f % 2:
                turn(f)   # the same instances again: the update of the slot the previous frame still reads
            sc.render_frame(fresh_core, converge=1)
        return fresh_core.accumulator(), fresh_core.ray_counts()

    for n in (1, 2, 3, 5):
        for double in (False, True):
            a, ca = run(n, 0, double)
            assert np.any(a[..., :3] != 0)
            for overlap in (1, 2):
                b, cb = run(n, overlap, double)
                assert np.array_equal(ca, cb), (n, double, overlap, ca[:6], cb[:6])
                assert rel_l2(b[..., :3], a[..., :3]) <= 1e-6, (n, double, overlap)
                assert np.array_equal(a[..., 3], b[..., 3]), (n, double, overlap)


@pytest.mark.parametrize("gpu_build", [0, 1])
def test_animated_frames_with_new_geometry(gpu_build):
    """Instances moved every frame (instance-only UpdateToplevel: the TLAS slot no frame in flight reads, on the ahead
    stream) and, midway, a new mesh and instance (SetGeometry: new BLAS arrays, the frame waits for everything queued;
    gpuBuild 1: the GPU builder, whose scratch the queued TLAS builds share).  Frames queued back to back equal the
    same frames serialised (frameOverlap 0): the same ray counts, the accumulator to float summation order."""
    w, h = 96, 64
    sc = scene.instanced_scene(meshes=4, tris_per_mesh=4000, width=w, height=h, grid=2, spacing=10.0)
    sc.sky = scene.gradient_sky(64, 32)
    extra = scene.random_triangles(3000, seed=99)

    def run(overlap):
        core = RenderCore(device=0)   # each run from a fresh core (the first one leaves its extra mesh behind)
        core.setting("gpuBuild", gpu_build)
        core.setting("frameOverlap", overlap)
        sc2 = scene.instanced_scene(meshes=4, tris_per_mesh=4000, width=w, height=h, grid=2, spacing=10.0)
        sc2.sky = sc.sky
        sc2.load_into(core)
        core.set_target(w, h, 1)
        core.setting("maxPathLength", 3)
        n = len(sc2.instances)
        for f in range(6):
            scene.animate_instances(sc2, f)
            for k, (mesh, T) in enumerate(sc2.instances):
                core.set_instance(k, mesh, T)
            if f == 3:
                core.set_geometry(len(sc2.meshes), extra)
                T = np.eye(4, dtype=np.float32)
                T[1, 3] = 3.0
                core.set_instance(n, len(sc2.meshes), T)
            core.update_toplevel()
            sc2.render_frame(core, converge=1 if f == 0 else 0)
        out = core.accumulator(), core.ray_counts()
        core.close()
        return out

    a, ca = run(0)
    assert np.any(a[..., :3] != 0)
    for overlap in (1, 2):
        b, cb = run(overlap)
        assert np.array_equal(ca, cb), (overlap, ca[:6], cb[:6])
        assert rel_l2(b[..., :3], a[..., :3]) <= 1e-6, overlap


@pytest.mark.parametrize("packets", [-1, 0])
def test_early_frame_ending_before_its_tail(fresh_core, packets):
    """with the path tail from bounce 4, an early frame (its first shade launch on the ahead stream, beside the
    previous frame's tail) whose paths all end at their first vertex (every primary ray misses: the camera looks away from
    the room) leaves the bounce loop before the shade launch before its tail.  Its overlap event, which the next frames'
    counter resets and primary launches order themselves after, must then be a core-stream event behind the previous
    frame's finalize (RenderCore::Render, PathStreams::evEarlyEnd), not the early shade.  Frames that alternate between the
    room and the empty view, queued back to back, equal the same frames serialised (frameOverlap 0)."""
    w, h = 96, 64
    sc = scene.room_scene(40000, w, h)
    room_view = sc.view
    away = scene.camera_view((0, 6, 200), (0, 0, 1), fov_deg=60, aspect=w / h, focal=5, pixel_height=h)
    fresh_core.setting("packetPrimary", packets)
    sc.load_into(fresh_core)
    fresh_core.set_target(w, h, 1)
    fresh_core.setting("maxPathLength", 6)
    fresh_core.setting("pathTail", 4)
    views = [room_view, away, away, room_view, away, room_view, room_view, away]

    def run(overlap):
        fresh_core.setting("frameOverlap", overlap)
        for f, v in enumerate(views):
            sc.render_frame(fresh_core, converge=1 if f == 0 else 0, view=v)
        return fresh_core.accumulator(), fresh_core.ray_counts()

    a, ca = run(0)
    assert np.any(a[..., :3] != 0)
    for overlap in (1, 2):
        b, cb = run(overlap)
        assert np.array_equal(ca, cb), overlap
        assert rel_l2(b[..., :3], a[..., :3]) <= 1e-6, overlap
        assert np.array_equal(a[..., 3], b[..., 3]), overlap
