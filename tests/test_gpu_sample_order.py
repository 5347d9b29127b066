"""GPU parity of the sample-interleaved primary ray order (setting sampleInterleave, k_camera): with spp > 1
the samples of an 8x8 pixel block are stored in consecutive waves instead of a whole frame of rays
apart.  Storage order only: every path keeps its pixel, sample index and random numbers (camera.h:48-70),
so per-bounce ray counts are identical and the accumulator equals the sample-major order's to float
summation order, and the CPU oracle's within the frame tolerance.  Covers frames whose height leaves
rows outside the full 8-row blocks, widths that are not a multiple of 8 (row-major storage) and band
tiles.  Off by default: config 5 (8 spp) measured no faster (profiles/r02zl_ab_sample_interleave.txt)."""
import numpy as np
import pytest

from lighthouse2_amd import parallel, scene
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("w,h,spp,bands", [(96, 60, 3, False), (100, 56, 2, False), (128, 72, 4, True)])
def test_sample_interleave_frame_parity(fresh_core, w, h, spp, bands):
    sc = scene.room_scene(20000, w, h)
    sc.load_into(fresh_core)
    fresh_core.set_target(w, h, spp)
    fresh_core.setting("maxPathLength", 3)
    if bands:
        fresh_core.set_tile_bands(1, 2, parallel.BAND)
    fresh_core.setting("sampleInterleave", 1)
    sc.render_frame(fresh_core)
    a1, c1 = fresh_core.accumulator(), fresh_core.ray_counts()
    fresh_core.setting("sampleInterleave", 0)
    sc.render_frame(fresh_core)
    a0, c0 = fresh_core.accumulator(), fresh_core.ray_counts()
    assert np.array_equal(c1, c0)
    assert rel_l2(a1[..., :3], a0[..., :3]) <= 1e-6
    if not bands:
        o = Oracle()
        sc.load_into(o)
        o.set_target(w, h, spp)
        o.setting("maxPathLength", 3)
        sc.render_frame(o)
        assert np.array_equal(c1, o.ray_counts())
        assert rel_l2(a1[..., :3], o.accumulator()[..., :3]) <= 1e-4
