"""The oracle pinned to the reference: the compiled RenderCore_Bart traversal (golden sample in
tests/golden/bart_config2_sample.npz, regenerated from /root/reference by tools/make_fixtures.py)
and regression goldens of whole oracle frames."""
import pathlib

import numpy as np
import pytest

from lighthouse2_amd import abi, scene
from oracle.oracle import Oracle

GOLD = pathlib.Path(__file__).resolve().parent / "golden"
REF_LIB = pathlib.Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "libbart_ref.so"


@pytest.fixture(scope="module")
def config2_oracle():
    sc = scene.config2_scene(n=100_000)
    o = Oracle(threads=8)
    sc.load_into(o)
    o.set_target(1920, 1080, 1)
    o.setting("epsilon", 1e-4)
    return sc, o


def test_oracle_matches_reference_traversal_sample(config2_oracle):
    """Closest-hit distance and face normal of the oracle vs RenderCore_Bart BVH2::Traverse on the
    64x36 golden sample of config-2 primary rays.  Bart normalises the direction again
    (common.h:10) and computes 1/a in double (common.h:33), so t agrees to a few ulp."""
    sc, o = config2_oracle
    g = np.load(GOLD / "bart_config2_sample.npz")
    n = len(g["org"])
    O4 = np.concatenate([g["org"], np.full((n, 1), 1e-4, np.float32)], 1)
    D4 = np.concatenate([g["dir"], np.full((n, 1), 1e34, np.float32)], 1)
    hits = o.trace_closest(O4, D4)
    ohit = hits[:, 1] != 0xFFFFFFFF
    bhit = g["t"] < 1e30
    assert (ohit == bhit).mean() >= 0.999
    both = ohit & bhit
    t_o = hits[both, 0].view(np.float32)
    t_b = g["t"][both]
    assert np.max(np.abs(t_o - t_b) / t_b) < 1e-5
    tris = sc.meshes[0]
    tri = hits[both, 1].astype(np.int64)
    N = np.stack([tris[tri, abi.TRI["Nx"]], tris[tri, abi.TRI["Ny"]], tris[tri, abi.TRI["Nz"]]], 1)
    assert np.mean(np.all(np.abs(N - g["normal"][both]) < 1e-6, axis=1)) >= 0.999


def test_oracle_visit_model_fixture(config2_oracle):
    """The n_node / n_tri model bench.py prices traffic with (tests/golden/config2_visits.json)."""
    import json
    sc, o = config2_oracle
    fix = json.loads((GOLD / "config2_visits.json").read_text())
    O4, D4, _ = o.generate_eye_rays(sc.view, 0, 0)
    sel = slice(0, None, 97)
    hits, vis = o.trace_closest(O4[sel], D4[sel], visits=True)
    assert abs(vis[:, 0].mean() - fix["mean_node_records"]) / fix["mean_node_records"] < 0.03
    assert abs(vis[:, 1].mean() - fix["mean_tri_tests"]) / fix["mean_tri_tests"] < 0.05


@pytest.mark.skipif(not REF_LIB.exists(), reason="reference traversal not built")
def test_oracle_matches_compiled_reference_on_random_rays():
    import ctypes as C
    L = C.CDLL(str(REF_LIB))
    L.bart_build.restype = C.c_void_p
    L.bart_build.argtypes = [C.c_void_p, C.c_int]
    L.bart_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
    tris = scene.random_triangles(20000, seed=99)
    h = L.bart_build(tris.ctypes.data, len(tris))
    rng = np.random.default_rng(5)
    n = 20000
    org = (rng.normal(size=(n, 3)) * 8).astype(np.float32)
    d = (rng.uniform(-3, 3, (n, 3)) - org).astype(np.float32)
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    out = np.zeros((n, 4), np.float32)
    L.bart_trace(h, org.ctypes.data, d.ctypes.data, n, out.ctypes.data, None, 4)
    o = Oracle(threads=4)
    o.set_materials([abi.make_material()])
    o.set_geometry(0, tris)
    o.set_instance(0, 0, None)
    o.update_toplevel()
    hits = o.trace_closest(np.concatenate([org, np.full((n, 1), 1e-4, np.float32)], 1),
                           np.concatenate([d, np.full((n, 1), 1e4, np.float32)], 1))
    ohit = hits[:, 1] != 0xFFFFFFFF
    bhit = out[:, 0] < 1e30
    assert (ohit == bhit).mean() >= 0.999
    both = ohit & bhit
    rel = np.abs(hits[both, 0].view(np.float32) - out[both, 0]) / out[both, 0]
    assert np.mean(rel < 1e-5) >= 0.999


@pytest.mark.parametrize("name,make", [
    ("config2_light_96x54", lambda: scene.config2_scene(n=5000, width=96, height=54, sky=True, light=True)),
    ("room_96x54", lambda: scene.room_scene(8000, 96, 54)),
    ("textured_96x54", lambda: scene.textured_scene(96, 54, tess=8))])
def test_oracle_frame_regression(name, make):
    g = np.load(GOLD / "oracle_frames.npz")
    sc = make()
    o = Oracle(threads=8)
    sc.load_into(o)
    o.set_target(96, 54, 1)
    sc.render_frame(o)
    assert np.array_equal(o.ray_counts(), g[name + "_counts"])
    assert np.array_equal(o.accumulator(), g[name + "_acc"])
