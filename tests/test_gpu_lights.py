"""GPU parity of every light type: point, spot and directional lights, alone and mixed with area lights,
rendered by the HIP core through the C-ABI against the CPU oracle.

The reference paths (CUDA/shared_kernel_code/lights_shared.h:36-261, RenderCore_OptixPrime_B/kernels/pathtracer.h:140-208):
NEE picks a light by its potential (RandomPointOnLight), so point and directional lights take part only with a non-zero
energy; spot lights always (their potential is the radiance sum).  A path that hits an area light after a diffuse bounce is
weighted by LightPickProb, whose sum runs over the potentials of every light type.  An unchanged RenderSystem reaches these
branches through SynchronizeLights -> SetLights (rendersystem.cpp:181-204); its conversions leave point / directional energy
at 0 (host_light.h:61, 103), as the "rendersystem" cases reproduce, and apps/ai_debugger/main.cpp:63 adds a directional
light (-1, -1, -1), radiance 255.  Bar: identical per-bounce and shadow ray counts, accumulator rel-L2 <= 1e-4 (north_star),
over two converging frames; the room cases run the default path tail (bounces 3-4 in k_trace_path4d) and the shadow-ray
launches beside it."""
import numpy as np
import pytest

from lighthouse2_amd import scene
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

REL_L2_TOL = 1e-4


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _spot(pos, aim, inner, outer, rad):
    return scene.spot_light(pos, scene._norm(scene._f3(*aim)), inner, outer, rad)


def _scene(kind, w, h):
    """(scene, maxPathLength, shadow rays expected)"""
    point = scene.point_light((2, 12, 1), (400, 380, 300), energy=1080.0)
    point0 = scene.point_light((-6, 10, -2), (300, 300, 300))                     # RenderSystem's conversion: energy 0
    spot = _spot((-8, 15, 0), (0.2, -1, 0.1), 0.95, 0.8, (900, 800, 600))         # a cone with a soft edge
    dirl = scene.directional_light(scene._norm(scene._f3(0.3, -1, 0.2)), (3, 3, 2.5), energy=8.5)
    if kind in ("point", "spot", "room_mixed", "room_rendersystem"):
        sc = scene.room_scene(40000, w, h)
        if kind == "point":
            sc.area_lights, sc.point_lights = [], [point]
        elif kind == "spot":
            sc.area_lights, sc.spot_lights = [], [spot, _spot((9, 14, -4), (-0.3, -1, 0.4), 0.9, 0.89, (200, 400, 200))]
        elif kind == "room_mixed":                                                  # all four types, the area lights first
            sc.point_lights, sc.spot_lights, sc.dir_lights = [point, point0], [spot], [dirl]
        else:                                                                       # as an unchanged RenderSystem hands them over
            sc.point_lights, sc.spot_lights = [point0], [spot]
            sc.dir_lights = [scene.directional_light((-1, -1, -1), (255, 255, 255))]
        return sc, 4, True
    sc = scene.config2_scene(n=20000, width=w, height=h, sky=True, light=kind == "open_mixed")
    if kind == "dir":
        sc.dir_lights = [dirl]
    elif kind == "open_mixed":
        sc.point_lights = [scene.point_light((0, 6, -6), (60, 60, 50), energy=170.0)]
        sc.spot_lights = [_spot((3, 8, -3), (-0.2, -1, 0.3), 0.9, 0.7, (200, 150, 100))]
        sc.dir_lights = [dirl, scene.directional_light(scene._norm(scene._f3(-0.5, -1, -0.1)), (1, 1.5, 2), energy=4.5)]
    else:   # "ai_debugger": the only light is the directional light of apps/ai_debugger/main.cpp:63, energy 0: no NEE at all
        sc.dir_lights = [scene.directional_light((-1, -1, -1), (255, 255, 255))]
        return sc, 2, False
    return sc, 2, True


@pytest.mark.parametrize("kind", ["point", "spot", "dir", "room_mixed", "open_mixed", "room_rendersystem", "ai_debugger"])
def test_light_types_frame_parity(fresh_core, kind):
    w, h = 128, 72
    sc, depth, shadows = _scene(kind, w, h)
    sc.load_into(fresh_core)
    fresh_core.set_target(w, h, 1)
    o = Oracle()
    sc.load_into(o)
    o.set_target(w, h, 1)
    for tgt in (fresh_core, o):
        tgt.setting("maxPathLength", depth)
    for f in range(2):
        sc.render_frame(fresh_core, converge=1 if f == 0 else 0)
        sc.render_frame(o, converge=1 if f == 0 else 0)
        cg, co = fresh_core.ray_counts(), o.ray_counts()
        assert np.array_equal(cg, co), (kind, f, cg[:6], cg[16], co[:6], co[16])
    assert (co[16] > 0) == shadows, (kind, co[16])
    ag, ao = fresh_core.accumulator(), o.accumulator()
    assert np.any(ao[..., :3] != 0)
    assert rel_l2(ag[..., :3], ao[..., :3]) <= REL_L2_TOL, (kind, rel_l2(ag[..., :3], ao[..., :3]))
    assert rel_l2(ag[..., 3], ao[..., 3]) <= 1e-6


def test_delta_lights_contribute(fresh_core):
    """The delta lights really light the frame: the room lit by a point light (energy > 0) is brighter than the same room
    whose point light has RenderSystem's energy 0 (never picked), on the GPU and in the oracle alike."""
    w, h = 96, 54
    res = []
    for energy in (1080.0, None):
        sc = scene.room_scene(30000, w, h)
        sc.area_lights = []
        sc.point_lights = [scene.point_light((2, 12, 1), (400, 380, 300), energy=energy)]
        sc.load_into(fresh_core)
        fresh_core.set_target(w, h, 1)
        fresh_core.setting("maxPathLength", 3)
        sc.render_frame(fresh_core, converge=1)
        res.append((fresh_core.accumulator()[..., :3].sum(), fresh_core.ray_counts()[16]))
    (lit, shadow_lit), (dark, shadow_dark) = res
    assert shadow_lit > 0 and shadow_dark == 0
    assert lit > 1.5 * dark
