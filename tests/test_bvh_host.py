"""Host-side invariants of the BLAS builder (lighthouse2_amd/csrc/bvh_build.cpp) on the CPU: tools/bvh_check.cpp builds
a config-2-density triangle soup and a grid of small triangles with plain binned SAH and with spatial splits (SBVH at
the default threshold 1e-3, at 1e-5, and only in nodes of >= 64 references), then checks that every triangle is in a
leaf, that sample points on every triangle (vertices, edge midpoints, seeded interior points) reach a leaf holding it
through closed child boxes that contain them (the spatial splits' clipped reference boxes still cover their triangle),
and that the reported depth bounds the real one.  The GPU parity tests check the hits on such trees
(test_gpu_parity.py::test_spatial_splits_bitexact); this one needs no GPU."""
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_bvh_builder_invariants(tmp_path):
    exe = tmp_path / "bvh_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", str(ROOT / "tools" / "bvh_check.cpp"),
                    str(ROOT / "lighthouse2_amd" / "csrc" / "bvh_build.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "20000"], capture_output=True, text=True, timeout=300)
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert r.returncode == 0 and not any("FAIL" in l for l in lines), r.stdout
    builds = [l for l in lines if l.endswith(" ok")]
    assert len(builds) == 8, r.stdout
    # the soup's spatial splits do add references (the case the coverage check is for)
    soup = {l.split(":")[0]: int(l.split("refs ")[1].split()[0]) for l in builds if l.startswith("soup")}
    assert soup["soup sbvh 1e-3"] > 1.2 * soup["soup sah"], soup
