"""The drop-in boundary: type layouts, vtable order and exported symbols of libRenderCore_MI355X.so.

Checks (CPU only, no GPU calls):
  * the Python ctypes mirror (lighthouse2_amd/abi.py) has the reference sizes/offsets;
  * include/lh2_core_types.h compiled with gcc gives the same numbers;
  * when /root/reference is present: the REFERENCE headers compiled with g++ give the same numbers
    and CoreAPI_Base's virtual slot order equals include/lh2_core_api.hpp's;
  * the library loads without a GPU and exports every function include/lh2_rendercore.h declares.
"""
import ctypes as C
import pathlib
import re
import subprocess

import pytest

from lighthouse2_amd import abi

ROOT = pathlib.Path(__file__).resolve().parents[1]
REF = pathlib.Path("/root/reference/lib")

FIELDS = {   # (struct, field) -> offset, from the reference layout
    ("CoreTri", "material"): 28, ("CoreTri", "Nx"): 44, ("CoreTri", "alpha"): 112, ("CoreTri", "vertex0"): 128,
    ("CoreTri", "vertex2"): 160, ("CoreMaterial", "flags"): 160, ("CoreMaterial", "absorption"): 168,
    ("CoreMaterial", "metallic"): 208, ("CoreMaterial", "roughness"): 304, ("CoreMaterial", "eta"): 560,
    ("CoreMaterial", "ior"): 656, ("CoreStats", "renderTime"): 52, ("CoreStats", "traceTime0"): 60,
    ("CoreStats", "probedDist"): 100, ("CoreLightTri", "vertex0"): 48, ("CoreLightTri", "instIdx"): 76,
    ("ViewPyramid", "aperture"): 48, ("ViewPyramid", "distortion"): 64,
}
PY_TYPES = {"CoreMaterial": abi.CoreMaterial, "CoreStats": abi.CoreStats, "CoreLightTri": abi.CoreLightTri,
            "ViewPyramid": abi.ViewPyramid, "CorePointLight": abi.CorePointLight, "CoreSpotLight": abi.CoreSpotLight,
            "CoreDirectionalLight": abi.CoreDirectionalLight, "Vec3Value": abi.Vec3Value,
            "ScalarValue": abi.ScalarValue, "GLTexture": abi.GLTexture, "CoreTexDesc": abi.CoreTexDesc}


def test_python_mirror_sizes_and_offsets():
    for name, cls in PY_TYPES.items():
        assert C.sizeof(cls) == abi.EXPECTED_SIZES[name], name
    assert abi.TRI_WORDS * 4 == abi.EXPECTED_SIZES["CoreTri"]
    for (s, f), off in FIELDS.items():
        if s == "CoreTri":
            assert abi.TRI[f] * 4 == off, (s, f)
        else:
            assert getattr(PY_TYPES[s], f).offset == off, (s, f)


def _probe(tmp_path, src, compiler, flags):
    c = tmp_path / "probe.cpp"
    c.write_text(src)
    exe = tmp_path / "probe"
    subprocess.run([compiler, *flags, str(c), "-o", str(exe)], check=True, capture_output=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return dict(line.split() for line in out.strip().splitlines())


REF_NAMES = {"Vec3Value": "CoreMaterial::Vec3Value", "ScalarValue": "CoreMaterial::ScalarValue"}


def _probe_src(prefix):
    def nm(n):
        return REF_NAMES.get(n, n) if prefix == "" else prefix + n
    lines = [f'printf("{n} %zu\\n", sizeof({nm(n)}));' for n in abi.EXPECTED_SIZES if n not in ("GLTexture", "CoreInstanceDesc")]
    lines += [f'printf("{s}.{f} %zu\\n", offsetof({nm(s)}, {f}));' for (s, f) in FIELDS]
    return "\n".join(lines)


def test_c_header_layout(tmp_path):
    src = "#include <cstdio>\n#include <cstddef>\n#include \"lh2_core_types.h\"\nint main(){\n" + _probe_src("lh2_") + \
          '\nprintf("CoreInstanceDesc %zu\\n", sizeof(lh2_CoreInstanceDesc));\nprintf("GLTexture %zu\\n", sizeof(lh2_GLTexture));\n}\n'
    got = _probe(tmp_path, src, "g++", ["-std=c++17", f"-I{ROOT / 'include'}"])
    for n, size in abi.EXPECTED_SIZES.items():
        assert int(got[n]) == size, n
    for (s, f), off in FIELDS.items():
        assert int(got[f"{s}.{f}"]) == off, (s, f)


REF_FLAGS = ["-std=c++17", "-w", "-include", "cfloat", "-DCOREDLL_EXPORTS", "-DWORD=unsigned short",
             "-DDWORD=unsigned int", "-DBYTE=unsigned char", "-DBOOL=int", "-DLONG=int", "-D__stdcall=",
             "-D__declspec(x)="] + [f"-I{REF / d}" for d in ("platform", "RenderSystem", "glad/include", "GLFW/include",
                                                              "half2.1.0", "zlib", "FreeImage/inc")]


@pytest.mark.skipif(not REF.exists(), reason="reference tree not present (GPU box)")
def test_reference_header_layout_matches(tmp_path):
    src = "#include \"platform.h\"\n#include \"core_api_base.h\"\n#include <cstddef>\nint main(){\n" + _probe_src("") + \
          '\nprintf("CoreInstanceDesc %zu\\n", sizeof(CoreInstanceDesc));\n}\n'
    # compile + link against nothing: the probe only needs the headers
    c = tmp_path / "ref_probe.cpp"
    c.write_text(src)
    exe = tmp_path / "ref_probe"
    r = subprocess.run(["g++", *REF_FLAGS, str(c), "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    got = dict(line.split() for line in out.strip().splitlines())
    for n, size in abi.EXPECTED_SIZES.items():
        if n in got:
            assert int(got[n]) == size, n
    for (s, f), off in FIELDS.items():
        assert int(got[f"{s}.{f}"]) == off, (s, f)


@pytest.mark.skipif(not REF.exists(), reason="reference tree not present (GPU box)")
def test_vtable_slot_order_matches_reference():
    """Same virtual function names in the same order as RenderSystem/core_api_base.h:84-113."""
    def strip(t):
        return re.sub(r"//[^\n]*", "", re.sub(r"/\*.*?\*/", "", t, flags=re.S))
    ref = strip((REF / "RenderSystem" / "core_api_base.h").read_text())
    ours = strip((ROOT / "include" / "lh2_core_api.hpp").read_text())
    pat = re.compile(r"virtual\s+[\w:<>]+\s*\*?\s*(\w+)\s*\(")
    ref_names = pat.findall(ref)
    our_names = pat.findall(ours)
    assert ref_names == our_names and len(ours) > 0 and len(our_names) == 14


def _declared_functions():
    hdr = (ROOT / "include" / "lh2_rendercore.h").read_text()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(lh2_\w+)\s*\(", hdr, re.M)))


def test_library_loads_and_exports_every_declared_symbol():
    lib = C.CDLL(str(ROOT / "lighthouse2_amd" / "libRenderCore_MI355X.so"))
    names = _declared_functions() + ["CreateCore", "DestroyCore"]
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
    lib.lh2_version.restype = C.c_char_p
    assert b"gfx950" in lib.lh2_version()


def test_library_exports_nothing_else():
    out = subprocess.run(["nm", "-D", "--defined-only", str(ROOT / "lighthouse2_amd" / "libRenderCore_MI355X.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert exported == set(_declared_functions()) | {"CreateCore", "DestroyCore"}


def test_code_object_targets_gfx950_only():
    blob = (ROOT / "lighthouse2_amd" / "libRenderCore_MI355X.so").read_bytes()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}
