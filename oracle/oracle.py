"""ctypes binding of the CPU oracle (oracle/liboracle.so) - TEST INFRASTRUCTURE ONLY.

The oracle is the parity checker of the MI355X render core: only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module.  Its method names match
lighthouse2_amd.core.RenderCore so that lighthouse2_amd.scene.Scene.load_into / render_frame drive
both the same way (the RenderSystem call order).
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib
import subprocess

import numpy as np

from lighthouse2_amd import abi

HERE = pathlib.Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
BLUENOISE = HERE.parent / "lighthouse2_amd" / "data" / "bluenoise.bin"

_P = C.c_void_p
_F = C.POINTER(C.c_float)
_U = C.POINTER(C.c_uint32)


class OracleStats(C.Structure):
    _fields_ = [("rayCount", C.c_uint32 * 16), ("shadowRays", C.c_uint32), ("maxPathLength", C.c_uint32),
                ("probedInstid", C.c_int), ("probedTriid", C.c_int), ("probedDist", C.c_float)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        L.orc_create.restype = _P
        sig = {
            "orc_destroy": [_P], "orc_set_bluenoise": [_P, C.POINTER(C.c_uint8)], "orc_set_max_path_length": [_P, C.c_int],
            "orc_set_geometry": [_P, C.c_int, _P, C.c_int], "orc_set_geometry_many": [_P, C.c_int, C.c_int, _P, _P, C.c_int], "orc_set_instance": [_P, C.c_int, C.c_int, _F],
            "orc_update_toplevel": [_P], "orc_set_materials": [_P, _P, C.c_int],
            "orc_set_lights": [_P, _P, C.c_int, _P, C.c_int, _P, C.c_int, _P, C.c_int],
            "orc_set_sky": [_P, _F, C.c_int, C.c_int], "orc_set_textures": [_P, _P, C.c_int],
            "orc_fetch_texel": [_P, C.c_int, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, C.c_float, C.c_int, _F], "orc_setting": [_P, C.c_char_p, C.c_float],
            "orc_set_target": [_P, C.c_int, C.c_int, C.c_int], "orc_set_probe": [_P, C.c_int, C.c_int],
            "orc_set_tile": [_P, C.c_int, C.c_int], "orc_set_tile_bands": [_P, C.c_int, C.c_int, C.c_int],
            "orc_render": [_P, C.POINTER(abi.ViewPyramid), C.c_int, C.c_int], "orc_get_accumulator": [_P, _F],
            "orc_get_stats": [_P, C.POINTER(OracleStats)],
            "orc_generate_eye_rays": [_P, C.POINTER(abi.ViewPyramid), C.c_uint32, C.c_int, _F, _F, _F],
            "orc_trace_closest": [_P, _F, _F, C.c_int, _U, _U, C.c_int], "orc_trace_any": [_P, _F, _F, C.c_int, _U],
            "orc_unpack_normal": [C.c_uint32, _F], "orc_mat4_inverse": [_F, _F],
            "orc_detmath_eval": [C.c_int, _F, _F, C.c_int, _F], "orc_debug_pixel": [_P, C.c_int, C.c_int],
        }
        for k, v in sig.items():
            getattr(L, k).argtypes = v
            getattr(L, k).restype = None
        L.orc_fetch_texel.restype = C.c_int
        L.orc_debug_log.argtypes = [_P, _F, C.c_int]
        L.orc_debug_log.restype = C.c_int
        L.orc_samples_taken.argtypes = [_P]
        L.orc_samples_taken.restype = C.c_int
        for k in ("orc_wanghash", "orc_xorshift"):
            getattr(L, k).argtypes = [C.c_uint32]
            getattr(L, k).restype = C.c_uint32
        L.orc_bluenoise.argtypes = [_P, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_bluenoise.restype = C.c_float
        L.orc_pack_normal.argtypes = [C.c_float] * 3
        L.orc_pack_normal.restype = C.c_uint32
        L.orc_light_potential.argtypes = [_P, C.c_int, _F, _F, _F, _F]
        L.orc_light_potential.restype = C.c_float
        L.orc_light_pick_prob.argtypes = [_P, C.c_int, _F, _F, _F]
        L.orc_light_pick_prob.restype = C.c_float
        L.orc_random_barycentrics.argtypes = [C.c_float, _F]
        L.orc_random_barycentrics.restype = None
        L.orc_random_point_on_light.argtypes = [_P, C.c_float, C.c_float, _F, _F, _F]
        L.orc_random_point_on_light.restype = None
        _lib = L
    return _lib


def _fp(a):
    return a.ctypes.data_as(_F)


def _up(a):
    return a.ctypes.data_as(_U)


class Oracle:
    """CPU restatement of RenderCore_OptixPrime_B (see oracle/pt_oracle.c)."""

    def __init__(self, threads: int | None = None):
        self.L = lib()
        self.o = self.L.orc_create()
        bn = np.fromfile(BLUENOISE, dtype=np.uint8)
        assert bn.size == 65536 * 5
        self._bn = bn
        self.L.orc_set_bluenoise(self.o, bn.ctypes.data_as(C.POINTER(C.c_uint8)))
        self.threads = threads or max(1, min(16, os.cpu_count() or 1))
        self.w = self.h = 0
        self.spp = 1

    def close(self):
        if self.o:
            self.L.orc_destroy(self.o)
            self.o = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # CoreAPI-shaped methods -----------------------------------------------------------
    def set_target(self, w, h, spp=1):
        self.w, self.h, self.spp = w, h, spp
        self.L.orc_set_target(self.o, w, h, spp)

    def setting(self, name, value):
        self.L.orc_setting(self.o, name.encode(), float(value))

    def set_probe(self, x, y):
        self.L.orc_set_probe(self.o, x, y)

    def debug_pixel(self, px, cap=256):
        """Diagnostics: the next renders log pixel px's path vertices and shadow rays (debug_log)."""
        self.L.orc_debug_pixel(self.o, int(px), int(cap))

    def debug_log(self, cap=256):
        """Records of debug_pixel: float32 (n, 16); kind 0 = vertex [kind, pathLength, hit t, tri (bits),
        inst (bits), O, D, tmin, tmax], kind 1 = shadow ray [kind, pathLength, occluded, O, D, tmax, rgb]."""
        out = np.zeros((cap, 16), np.float32)
        n = self.L.orc_debug_log(self.o, _fp(out), cap)
        return out[:n]

    def set_tile(self, y0, y1):
        self.L.orc_set_tile(self.o, y0, y1)

    def set_tile_bands(self, rank, nranks, band):
        self.L.orc_set_tile_bands(self.o, rank, nranks, band)

    def set_materials(self, mats):
        self._mats = abi.material_array(mats)
        self.L.orc_set_materials(self.o, C.cast(self._mats, _P), len(mats))

    def set_lights(self, area=(), point=(), spot=(), directional=()):
        def carr(cls, items):
            a = (cls * max(1, len(items)))()
            for i, it in enumerate(items):
                a[i] = it
            return a
        a, p, s, d = carr(abi.CoreLightTri, area), carr(abi.CorePointLight, point), carr(abi.CoreSpotLight, spot), \
            carr(abi.CoreDirectionalLight, directional)
        self.L.orc_set_lights(self.o, C.cast(a, _P), len(area), C.cast(p, _P), len(point), C.cast(s, _P), len(spot),
                              C.cast(d, _P), len(directional))

    def set_textures(self, textures):
        self._tex_keep = [np.ascontiguousarray(t.pixels) for t in textures]
        arr = (abi.CoreTexDesc * max(1, len(textures)))()
        for i, t in enumerate(textures):
            arr[i] = t.desc(self._tex_keep[i])
        self.L.orc_set_textures(self.o, C.cast(arr, _P), len(textures))

    def fetch_texel(self, storage, u, v, offset, w, h, lam=0.0, trilinear=False):
        out = np.zeros(4, np.float32)
        assert self.L.orc_fetch_texel(self.o, storage, u, v, offset, w, h, lam, int(trilinear), _fp(out)) == 0
        return out

    def set_sky(self, rgb):
        rgb = np.ascontiguousarray(rgb, np.float32)
        self.L.orc_set_sky(self.o, _fp(rgb), rgb.shape[1], rgb.shape[0])

    def set_geometry(self, idx, tris):
        tris = np.ascontiguousarray(tris, np.float32)
        self.L.orc_set_geometry(self.o, idx, tris.ctypes.data_as(_P), len(tris))

    def set_geometries(self, meshes, first=0):
        """SetGeometry for every mesh, the per-mesh builds spread over the oracle's threads."""
        keep = [np.ascontiguousarray(m, np.float32) for m in meshes]
        ptrs = (C.c_void_p * max(1, len(keep)))(*[k.ctypes.data for k in keep])
        counts = np.array([len(k) for k in keep] or [0], np.int32)
        self.L.orc_set_geometry_many(self.o, int(first), len(keep), C.cast(ptrs, _P), counts.ctypes.data_as(_P),
                                     self.threads)

    def set_instance(self, idx, mesh, T=None):
        m = np.ascontiguousarray(np.eye(4, dtype=np.float32) if T is None else T, np.float32)
        self.L.orc_set_instance(self.o, idx, mesh, _fp(m))

    def update_toplevel(self):
        self.L.orc_update_toplevel(self.o)

    def render(self, view, converge=1):
        self.L.orc_render(self.o, C.byref(view), converge, self.threads)

    # results -------------------------------------------------------------------------
    def accumulator(self):
        out = np.zeros((self.h, self.w, 4), np.float32)
        self.L.orc_get_accumulator(self.o, _fp(out))
        return out

    def frame(self):
        st = self.L.orc_samples_taken(self.o)
        return self.accumulator() * np.float32(1.0 / st)

    def stats(self) -> OracleStats:
        s = OracleStats()
        self.L.orc_get_stats(self.o, C.byref(s))
        return s

    def ray_counts(self):
        s = self.stats()
        out = np.zeros(17, np.uint32)
        out[:16] = np.array(s.rayCount, np.uint32)
        out[16] = s.shadowRays
        return out

    def generate_eye_rays(self, view, R0, pass_):
        n = self.w * self.h * self.spp
        o = np.zeros((n, 4), np.float32)
        d = np.zeros((n, 4), np.float32)
        s = np.zeros((n, 8), np.float32)
        self.L.orc_generate_eye_rays(self.o, C.byref(view), R0 & 0xffffffff, pass_, _fp(o), _fp(d), _fp(s))
        return o, d, s

    def trace_closest(self, org, dirs, visits=False):
        o = np.ascontiguousarray(org, np.float32)
        d = np.ascontiguousarray(dirs, np.float32)
        n = len(o)
        hits = np.zeros((n, 4), np.uint32)
        vis = np.zeros((n, 2), np.uint32) if visits else None
        self.L.orc_trace_closest(self.o, _fp(o), _fp(d), n, _up(hits), _up(vis) if visits else None, self.threads)
        return (hits, vis) if visits else hits

    def trace_any(self, org, dirs):
        o = np.ascontiguousarray(org, np.float32)
        d = np.ascontiguousarray(dirs, np.float32)
        mask = np.zeros((len(o) + 31) // 32, np.uint32)
        self.L.orc_trace_any(self.o, _fp(o), _fp(d), len(o), _up(mask))
        return mask


def detmath(fn: int, x, y=None) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, np.float32)
    out = np.zeros_like(x)
    lib().orc_detmath_eval(fn, _fp(x), _fp(y), len(x), _fp(out))
    return out
