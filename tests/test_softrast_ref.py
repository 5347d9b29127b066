"""BASELINE config 1 plumbing: the reference CPU rasterizer (RenderCore_SoftRasterizer/rasterizer.cpp,
built from the reference sources by oracle/Makefile.ref) renders tinyapp's default scene
(scene.tinyapp_scene, tests/golden/config1_tinyapp.npz) headless.  CPU only; skipped where the reference was not built."""
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
LIB = ROOT / "oracle" / "_ref" / "libsoftrast_ref.so"
sys.path.insert(0, str(ROOT / "tools"))


@pytest.mark.skipif(not LIB.exists(), reason="oracle/_ref not built (needs /root/reference)")
def test_soft_rasterizer_renders_config1_scene():
    import config1_plumbing as c1
    from lighthouse2_amd import scene
    sc = scene.tinyapp_scene(160, 100)
    r = c1.soft_rasterizer(sc, 160, 100, seconds=0.2)
    assert r["frames"] >= 1
    assert r["covered_pixel_share"] > 0.08, r      # tinyapp's default camera: the diorama fills ~12 % of the view


@pytest.mark.skipif(not LIB.exists(), reason="oracle/_ref not built (needs /root/reference)")
def test_soft_rasterizer_library_needs_no_gl():
    """--gc-sections dropped every OpenGL / FreeImage / GLFW reference of platform/system.cpp."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--undefined-only", str(LIB)], capture_output=True, text=True, check=True).stdout
    syms = [line.split()[-1] for line in out.splitlines() if line.strip()]
    assert not [s for s in syms if s.startswith(("gl", "FreeImage", "_glfw"))], syms
