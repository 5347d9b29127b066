"""ctypes / numpy mirror of the RenderCore C-ABI types (include/lh2_core_types.h).

The sizes and offsets are those of the reference headers on x86-64 (see the citations in
include/lh2_core_types.h); tests/test_abi_layout.py checks this module, the C header and, when
/root/reference is present, the reference headers against each other.
"""
from __future__ import annotations

import ctypes as C

import numpy as np


class float3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class float2(C.Structure):
    _pack_ = 8
    _fields_ = [("x", C.c_float), ("y", C.c_float)]


class int2(C.Structure):
    _fields_ = [("x", C.c_int), ("y", C.c_int)]


class Vec3Value(C.Structure):
    _fields_ = [("value", float3), ("textureID", C.c_int), ("scale", C.c_float), ("_pad", C.c_uint32),
                ("uvscale", C.c_float * 2), ("uvoffset", C.c_float * 2)]


class ScalarValue(C.Structure):
    _fields_ = [("value", C.c_float), ("textureID", C.c_int), ("component", C.c_int), ("scale", C.c_float),
                ("uvscale", C.c_float * 2), ("uvoffset", C.c_float * 2)]


_SCALARS = ["metallic", "subsurface", "specular", "roughness", "specularTint", "anisotropic", "sheen",
            "sheenTint", "clearcoat", "clearcoatGloss", "transmission", "eta", "reflection", "refraction", "ior"]


class CoreMaterial(C.Structure):
    _fields_ = ([("color", Vec3Value), ("detailColor", Vec3Value), ("normals", Vec3Value),
                 ("detailNormals", Vec3Value), ("flags", C.c_uint32), ("_pad", C.c_uint32),
                 ("absorption", Vec3Value)] + [(n, ScalarValue) for n in _SCALARS])


class CoreLightTri(C.Structure):
    _fields_ = [("centre", float3), ("energy", C.c_float), ("N", float3), ("area", C.c_float),
                ("radiance", float3), ("dummy2", C.c_int), ("vertex0", float3), ("triIdx", C.c_int),
                ("vertex1", float3), ("instIdx", C.c_int), ("vertex2", float3), ("dummy1", C.c_int)]


class CorePointLight(C.Structure):
    _fields_ = [("position", float3), ("energy", C.c_float), ("radiance", float3), ("dummy", C.c_int)]


class CoreSpotLight(C.Structure):
    _fields_ = [("position", float3), ("cosInner", C.c_float), ("radiance", float3), ("cosOuter", C.c_float),
                ("direction", float3), ("dummy", C.c_int)]


class CoreDirectionalLight(C.Structure):
    _fields_ = [("direction", float3), ("energy", C.c_float), ("radiance", float3), ("dummy", C.c_int)]


class CoreTexDesc(C.Structure):
    """CoreTexDesc (common_classes.h:246-269, host layout): texel pointer + sizes; firstPixel is set by
    the core (rendercore.cpp:328)."""
    _fields_ = [("idata", C.c_void_p), ("width", C.c_uint32), ("height", C.c_uint32), ("flags", C.c_uint32),
                ("pixelCount", C.c_uint32), ("firstPixel", C.c_uint32), ("MIPlevels", C.c_uint32), ("storage", C.c_int32)]


class ViewPyramid(C.Structure):
    _fields_ = [("pos", float3), ("p1", float3), ("p2", float3), ("p3", float3), ("aperture", C.c_float),
                ("spreadAngle", C.c_float), ("imagePlane", C.c_float), ("focalDistance", C.c_float),
                ("distortion", C.c_float)]


class CoreStats(C.Structure):
    _fields_ = [("deviceName", C.c_char_p), ("SMcount", C.c_uint32), ("ccMajor", C.c_uint32),
                ("ccMinor", C.c_uint32), ("VRAM", C.c_uint32), ("argb32TexelCount", C.c_uint32),
                ("argb128TexelCount", C.c_uint32), ("nrm32TexelCount", C.c_uint32), ("bvhBuildTime", C.c_float),
                ("totalRays", C.c_uint32), ("totalExtensionRays", C.c_uint32), ("totalShadowRays", C.c_uint32),
                ("renderTime", C.c_float), ("primaryRayCount", C.c_uint32), ("traceTime0", C.c_float),
                ("bounce1RayCount", C.c_uint32), ("traceTime1", C.c_float), ("deepRayCount", C.c_uint32),
                ("traceTimeX", C.c_float), ("shadowTraceTime", C.c_float), ("shadeTime", C.c_float),
                ("filterTime", C.c_float), ("probedInstid", C.c_int), ("probedTriid", C.c_int),
                ("probedDist", C.c_float)]


class GLTexture(C.Structure):
    _fields_ = [("ID", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32)]


# --- CoreTri as a (N, 44) float32/uint32 record array (176 B per triangle) -------------------
TRI_WORDS = 44
TRI = dict(u=0, ltriIdx=3, v=4, material=7, vN0=8, Nx=11, vN1=12, Ny=15, vN2=16, Nz=19, T=20, area=23,
           B=24, invArea=27, alpha=28, LOD=31, vertex0=32, vertex1=36, vertex2=40)

EXPECTED_SIZES = {
    "CoreTri": 176, "CoreMaterial": 688, "Vec3Value": 40, "ScalarValue": 32, "CoreLightTri": 96,
    "CorePointLight": 32, "CoreSpotLight": 48, "CoreDirectionalLight": 32, "ViewPyramid": 68,
    "CoreStats": 104, "CoreTexDesc": 40, "CoreInstanceDesc": 80, "GLTexture": 12,
}


def new_tris(n: int) -> np.ndarray:
    """Zeroed CoreTri records with ltriIdx = -1, as the host-side CoreTri constructor does
    (common_classes.h:62)."""
    t = np.zeros((n, TRI_WORDS), dtype=np.float32)
    t.view(np.int32)[:, TRI["ltriIdx"]] = -1
    return t


def tris_from_vertices(v0: np.ndarray, v1: np.ndarray, v2: np.ndarray, material: np.ndarray | int,
                       vertex_normals: tuple[np.ndarray, np.ndarray, np.ndarray] | None = None) -> np.ndarray:
    """CoreTri records the way HostScene::AddTriToMesh builds them (host_scene.cpp:208-223):
    flat normal N = normalize(cross(v1 - v0, v2 - v0)) for the face and, unless `vertex_normals`
    (vN0, vN1, vN2 as HostMesh::LoadGeometryFromOBJ stores them, host_mesh.cpp:246-253) is given, all three vertices."""
    v0 = np.asarray(v0, np.float32)
    v1 = np.asarray(v1, np.float32)
    v2 = np.asarray(v2, np.float32)
    n = len(v0)
    t = new_tris(n)
    N = np.cross(v1 - v0, v2 - v0).astype(np.float32)
    ln = np.sqrt((N * N).sum(1, dtype=np.float32)).astype(np.float32)
    ln[ln == 0] = 1
    N = (N * (np.float32(1) / ln)[:, None]).astype(np.float32)
    for i, k in enumerate(("vN0", "vN1", "vN2")):
        t[:, TRI[k]:TRI[k] + 3] = N if vertex_normals is None else np.asarray(vertex_normals[i], np.float32)
    t[:, TRI["Nx"]] = N[:, 0]
    t[:, TRI["Ny"]] = N[:, 1]
    t[:, TRI["Nz"]] = N[:, 2]
    t[:, TRI["vertex0"]:TRI["vertex0"] + 3] = v0
    t[:, TRI["vertex1"]:TRI["vertex1"] + 3] = v1
    t[:, TRI["vertex2"]:TRI["vertex2"] + 3] = v2
    t.view(np.uint32)[:, TRI["material"]] = np.asarray(material, np.uint32)
    # tangent frame without uvs: T = normalize(v1 - v0), B = normalize(cross(N, T))
    # (HostMesh::BuildFromIndexedData, host_mesh.cpp:562-564)
    T = (v1 - v0).astype(np.float32)
    lt = np.sqrt((T * T).sum(1, dtype=np.float32)).astype(np.float32)
    lt[lt == 0] = 1
    T = (T * (np.float32(1) / lt)[:, None]).astype(np.float32)
    B = np.cross(N, T).astype(np.float32)
    lb = np.sqrt((B * B).sum(1, dtype=np.float32)).astype(np.float32)
    lb[lb == 0] = 1
    B = (B * (np.float32(1) / lb)[:, None]).astype(np.float32)
    t[:, TRI["T"]:TRI["T"] + 3] = T
    t[:, TRI["B"]:TRI["B"] + 3] = B
    # triangle area (HostMesh::UpdateArea, Heron's formula, common_classes.h:83-90)
    a = np.linalg.norm(v1 - v0, axis=1).astype(np.float32)
    b = np.linalg.norm(v2 - v1, axis=1).astype(np.float32)
    c = np.linalg.norm(v0 - v2, axis=1).astype(np.float32)
    s = (a + b + c) * np.float32(0.5)
    t[:, TRI["area"]] = np.sqrt(np.maximum(s * (s - a) * (s - b) * (s - c), 0)).astype(np.float32)
    return t


def default_material() -> CoreMaterial:
    """HostMaterial defaults (host_material.h:34-116): colour 1, every other parameter 'not set'
    (value 1e-32, textureID -1), flags SMOOTH."""
    m = CoreMaterial()
    for f in ("color", "detailColor", "normals", "detailNormals", "absorption"):
        v = getattr(m, f)
        v.value = float3(1e-32, 1e-32, 1e-32)
        v.textureID = -1
        v.scale = 1
        v.uvscale[0] = v.uvscale[1] = 1
    m.color.value = float3(1, 1, 1)
    m.flags = 1
    for f in _SCALARS:
        s = getattr(m, f)
        s.value = 1e-32
        s.textureID = -1
        s.scale = 1
        s.uvscale[0] = s.uvscale[1] = 1
    return m


def make_material(color=(1, 1, 1), roughness=None, metallic=None, specular=None, transmission=None, eta=None,
                  absorption=None, sheen=None, clearcoat=None, clearcoatGloss=None, subsurface=None,
                  smooth: bool = True) -> CoreMaterial:
    m = default_material()
    m.color.value = float3(*color)
    for name, val in (("roughness", roughness), ("metallic", metallic), ("specular", specular),
                      ("transmission", transmission), ("eta", eta), ("sheen", sheen), ("clearcoat", clearcoat),
                      ("clearcoatGloss", clearcoatGloss), ("subsurface", subsurface)):
        if val is not None:
            getattr(m, name).value = float(val)
    if absorption is not None:
        m.absorption.value = float3(*absorption)
    m.flags = 1 if smooth else 0
    return m


def material_array(mats) -> C.Array:
    arr = (CoreMaterial * max(1, len(mats)))()
    for i, m in enumerate(mats):
        arr[i] = m
    return arr


def mat4_identity() -> np.ndarray:
    return np.eye(4, dtype=np.float32)
