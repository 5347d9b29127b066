"""Texture maps on the GPU (material_shared.h:99-171, sampling_shared.h:35-86):
trilinear diffuse + detail maps, alpha cut-outs (pathtracer.h:109-121 pass-through), NRM32 normal
map + detail normal map, roughness map, UV scale / offset, instanced with rotation and scale.
Bar: identical per-bounce ray counts (alpha decisions are exact) and accumulator rel-L2 <= 1e-4."""
import numpy as np
import pytest

from lighthouse2_amd import scene
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def _frames(core, sc, w, h, spp, frames, depth=16):
    sc.load_into(core)
    core.set_target(w, h, spp)
    core.setting("maxPathLength", depth)
    o = Oracle()
    sc.load_into(o)
    o.set_target(w, h, spp)
    o.setting("maxPathLength", depth)
    for f in range(frames):
        sc.render_frame(core, converge=1 if f == 0 else 0)
        sc.render_frame(o, converge=1 if f == 0 else 0)
        assert np.array_equal(core.ray_counts(), o.ray_counts()), (core.ray_counts(), o.ray_counts())
    ag, ao = core.accumulator(), o.accumulator()
    rel = float(np.linalg.norm(ag[..., :3] - ao[..., :3]) / np.linalg.norm(ao[..., :3]))
    assert rel <= 1e-4, rel
    return o.ray_counts()


@pytest.mark.parametrize("spp,frames,depth", [(1, 1, 16), (2, 2, 4)])
def test_textured_frame_parity(fresh_core, spp, frames, depth):
    w, h = 128, 72
    sc = scene.textured_scene(w, h, tess=12)
    counts = _frames(fresh_core, sc, w, h, spp, frames, depth)
    assert counts[2] > 0                      # alpha pass-through and specular chains reach bounce 3


def test_texture_descriptors_and_stats(fresh_core):
    sc = scene.textured_scene(64, 36, tess=6)
    sc.load_into(fresh_core)
    st = fresh_core.stats()
    argb = sum(t.pixels.size for t in sc.textures if t.storage == 0)
    nrm = sum(t.pixels.size for t in sc.textures if t.storage == 2)
    assert st.argb32TexelCount == max(16, argb) and st.nrm32TexelCount == max(16, nrm)
