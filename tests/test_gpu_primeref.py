"""PrimeRef validation mode: the RenderCore_PrimeRef path tracer
(kernels/pathtracer.h:44-165, Lambert bsdf.h:18-101: uniform random numbers, NEE without MIS,
Russian roulette at every vertex, MAXPATHLENGTH 64, per-bounce shadow passes) selected with the
setting "primeRef" on the same core and scene data.  Bar: identical per-bounce ray counts and shadow
ray totals, accumulator rel-L2 <= 1e-4 against the oracle's restatement."""
import numpy as np
import pytest

from lighthouse2_amd import scene
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,make,spp,frames", [
    ("room", lambda w, h: scene.room_scene(40000, w, h), 1, 1),
    ("config2_light", lambda w, h: scene.config2_scene(n=5000, width=w, height=h, sky=True, light=True), 2, 2),
    ("textured", lambda w, h: scene.textured_scene(w, h, tess=8), 1, 2)])
def test_primeref_frame_parity(fresh_core, name, make, spp, frames):
    w, h = 128, 72
    sc = make(w, h)
    sc.load_into(fresh_core)
    fresh_core.set_target(w, h, spp)
    fresh_core.setting("primeRef", 1)
    o = Oracle()
    sc.load_into(o)
    o.set_target(w, h, spp)
    o.setting("primeRef", 1)
    for f in range(frames):
        sc.render_frame(fresh_core, converge=1 if f == 0 else 0)
        sc.render_frame(o, converge=1 if f == 0 else 0)
        cg, co = fresh_core.ray_counts(), o.ray_counts()
        assert np.array_equal(cg, co), (cg, co)
    ag, ao = fresh_core.accumulator(), o.accumulator()
    rel = float(np.linalg.norm(ag[..., :3] - ao[..., :3]) / np.linalg.norm(ao[..., :3]))
    assert rel <= 1e-4, rel
    st = fresh_core.stats()
    assert st.totalShadowRays == int(co[16])


def test_primeref_differs_from_default(fresh_core):
    """The mode switch reaches the kernels: Russian roulette changes the bounce counts."""
    w, h = 96, 54
    sc = scene.room_scene(20000, w, h)
    sc.load_into(fresh_core)
    fresh_core.set_target(w, h, 1)
    sc.render_frame(fresh_core)
    c0 = fresh_core.ray_counts()
    fresh_core.setting("primeRef", 1)
    sc.render_frame(fresh_core)
    c1 = fresh_core.ray_counts()
    assert c0[0] == c1[0] and not np.array_equal(c0, c1)
