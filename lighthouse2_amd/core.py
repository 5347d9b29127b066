"""Python host binding of libRenderCore_MI355X.so (the ctypes stub a Lighthouse 2 maintainer would add).

Mirrors the reference CoreAPI_Base interface (lib/RenderSystem/core_api_base.h:84-113) method for
method, with the reference's call order (RenderSystem::SynchronizeSceneData, rendersystem.cpp:214-222).
Every call goes through the flat C-ABI of include/lh2_rendercore.h, which in turn calls the
CoreAPI_Base vtable of the core.  There is no fallback: if the library is missing or a call fails,
an exception is raised.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

import numpy as np

from . import abi

_LIB = None
LIB_PATH = pathlib.Path(__file__).resolve().parent / "libRenderCore_MI355X.so"

_P = C.c_void_p
_F = C.POINTER(C.c_float)
_U = C.POINTER(C.c_uint32)


class CoreError(RuntimeError):
    pass


def load_library(path: str | os.PathLike | None = None) -> C.CDLL:
    """Load the render core (fails loudly when the HIP library has not been built).

    When the process also uses PyTorch (bench.py, the distributed gather), import torch FIRST: its
    bundled libamdhip64.so carries the soname libamdhip64.so.7, which this library then binds to,
    so device pointers are shared by one HIP runtime."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = pathlib.Path(path) if path else pathlib.Path(os.environ.get("LH2_CORE_LIB", LIB_PATH))
    if not p.exists():
        raise CoreError(f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
    lib.lh2_version.restype = C.c_char_p
    lib.lh2_last_error.restype = C.c_char_p
    sig = {
        "lh2_set_device": [C.c_int],
        "lh2_core_new": [C.POINTER(_P)],
        "lh2_core_delete": [_P],
        "lh2_core_init": [_P],
        "lh2_core_get_stats": [_P, C.POINTER(abi.CoreStats)],
        "lh2_core_set_probe": [_P, C.c_int, C.c_int],
        "lh2_core_set_target": [_P, C.c_uint32, C.c_uint32, C.c_uint32],
        "lh2_core_setting": [_P, C.c_char_p, C.c_float],
        "lh2_core_get_setting": [_P, C.c_char_p, C.POINTER(C.c_float)],
        "lh2_core_render": [_P, C.POINTER(abi.ViewPyramid), C.c_int],
        "lh2_core_shutdown": [_P],
        "lh2_core_set_textures": [_P, _P, C.c_int],
        "lh2_core_set_materials": [_P, C.POINTER(abi.CoreMaterial), C.c_int],
        "lh2_core_set_lights": [_P, _P, C.c_int, _P, C.c_int, _P, C.c_int, _P, C.c_int],
        "lh2_core_set_sky": [_P, _F, C.c_uint32, C.c_uint32],
        "lh2_core_set_geometry": [_P, C.c_int, _F, C.c_int, C.c_int, _P, _U],
        "lh2_core_set_instance": [_P, C.c_int, C.c_int, _F],
        "lh2_core_update_toplevel": [_P],
        "lh2_core_set_tile": [_P, C.c_int, C.c_int],
        "lh2_core_set_tile_bands": [_P, C.c_int, C.c_int, C.c_int],
        "lh2_core_sync": [_P],
        "lh2_core_get_accumulator": [_P, _F],
        "lh2_core_get_frame": [_P, _F],
        "lh2_core_copy_accumulator_rows": [_P, _P, C.c_int, C.c_int],
        "lh2_core_ray_counts": [_P, _U],
        "lh2_core_pack_tile": [_P, _P],
        "lh2_core_copy_frame_async": [_P, _P],
        "lh2_core_pack_tile_ordered": [_P, _P, _P],
        "lh2_core_tile_rows": [_P, C.POINTER(C.c_int)],
        "lh2_core_stream": [_P, C.POINTER(_P)],
        "lh2_core_trace_closest": [_P, _F, _F, C.c_int, _U],
        "lh2_core_trace_any": [_P, _F, _F, C.c_int, _U],
        "lh2_core_trace_closest_device": [_P, _P, _P, C.c_int, _P, C.c_int, _F],
        "lh2_core_generate_eye_rays": [_P, C.POINTER(abi.ViewPyramid), C.c_uint32, C.c_int, _F, _F, _F],
        "lh2_core_scene_info": [_P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)],
        "lh2_xorshift_floats": [C.c_uint32, _F, C.c_uint64],
        "lh2_core_debug_shadow_rays": [_P, _F, _F, _F, C.c_int, C.POINTER(C.c_int)],
        "lh2_core_debug_bvh4": [_P, _F, C.c_void_p, C.c_int, C.POINTER(C.c_int)],
        "lh2_core_debug_poison_tlas": [_P, C.c_float],
    }
    for name, args in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_int
    if path is None:
        _LIB = lib
    return lib


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_F)


def _up(a: np.ndarray):
    return a.ctypes.data_as(_U)


class RenderCore:
    """One MI355X render core on the current (or given) HIP device."""

    def __init__(self, device: int | None = None, lib: C.CDLL | None = None):
        self.lib = lib or load_library()
        if device is not None:
            self._chk(self.lib.lh2_set_device(int(device)))
        h = _P()
        self._chk(self.lib.lh2_core_new(C.byref(h)))
        self.h = h
        self.w = self.h_ = 0
        self.spp = 1

    # --- plumbing ---------------------------------------------------------------------
    def _chk(self, rc: int) -> None:
        if rc != 0:
            raise CoreError(self.lib.lh2_last_error().decode())

    def close(self) -> None:
        if getattr(self, "h", None):
            self._chk(self.lib.lh2_core_delete(self.h))
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # --- CoreAPI_Base -----------------------------------------------------------------
    def set_target(self, width: int, height: int, spp: int = 1) -> None:
        self.w, self.h_, self.spp = int(width), int(height), int(spp)
        self._chk(self.lib.lh2_core_set_target(self.h, width, height, spp))

    def setting(self, name: str, value: float) -> None:
        self._chk(self.lib.lh2_core_setting(self.h, name.encode(), float(value)))

    def get_setting(self, name: str) -> float:
        v = C.c_float(0)
        self._chk(self.lib.lh2_core_get_setting(self.h, name.encode(), C.byref(v)))
        return v.value

    def set_probe(self, x: int, y: int) -> None:
        self._chk(self.lib.lh2_core_set_probe(self.h, int(x), int(y)))

    def set_textures(self, textures) -> None:
        """textures: scene.Texture list (RenderSystem order: before set_materials)."""
        self._tex_keep = [np.ascontiguousarray(t.pixels) for t in textures]
        arr = (abi.CoreTexDesc * max(1, len(textures)))()
        for i, t in enumerate(textures):
            arr[i] = t.desc(self._tex_keep[i])
        self._chk(self.lib.lh2_core_set_textures(self.h, C.cast(arr, _P), len(textures)))

    def set_materials(self, mats) -> None:
        arr = abi.material_array(mats)
        self._chk(self.lib.lh2_core_set_materials(self.h, arr, len(mats)))

    def set_lights(self, area=(), point=(), spot=(), directional=()) -> None:
        def carr(cls, items):
            a = (cls * max(1, len(items)))()
            for i, it in enumerate(items):
                a[i] = it
            return a, len(items)
        a, na = carr(abi.CoreLightTri, area)
        p, np_ = carr(abi.CorePointLight, point)
        s, ns = carr(abi.CoreSpotLight, spot)
        d, nd = carr(abi.CoreDirectionalLight, directional)
        self._chk(self.lib.lh2_core_set_lights(self.h, C.cast(a, _P), na, C.cast(p, _P), np_, C.cast(s, _P), ns,
                                               C.cast(d, _P), nd))

    def set_sky(self, rgb: np.ndarray) -> None:
        rgb = np.ascontiguousarray(rgb, dtype=np.float32)
        h, w = rgb.shape[:2]
        self._chk(self.lib.lh2_core_set_sky(self.h, _fp(rgb), w, h))

    def set_geometry(self, mesh_idx: int, tris: np.ndarray) -> None:
        tris = np.ascontiguousarray(tris, dtype=np.float32)
        assert tris.ndim == 2 and tris.shape[1] == abi.TRI_WORDS
        n = len(tris)
        verts = np.zeros((max(3 * n, 1), 4), np.float32)
        if n:
            verts[0::3, :3] = tris[:, 32:35]
            verts[1::3, :3] = tris[:, 36:39]
            verts[2::3, :3] = tris[:, 40:43]
            verts[:, 3] = 1
        self._chk(self.lib.lh2_core_set_geometry(self.h, int(mesh_idx), _fp(verts), 3 * n, n,
                                                 tris.ctypes.data_as(_P), None))

    def set_instance(self, idx: int, mesh_idx: int, transform: np.ndarray | None = None) -> None:
        m = np.ascontiguousarray(np.eye(4, dtype=np.float32) if transform is None else transform, dtype=np.float32)
        self._chk(self.lib.lh2_core_set_instance(self.h, int(idx), int(mesh_idx), _fp(m)))

    def update_toplevel(self) -> None:
        self._chk(self.lib.lh2_core_update_toplevel(self.h))

    def render(self, view: abi.ViewPyramid, converge: int = 1) -> None:
        self._chk(self.lib.lh2_core_render(self.h, C.byref(view), int(converge)))

    def stats(self) -> abi.CoreStats:
        s = abi.CoreStats()
        self._chk(self.lib.lh2_core_get_stats(self.h, C.byref(s)))
        return s

    # --- extensions -------------------------------------------------------------------
    def set_tile(self, y0: int, y1: int) -> None:
        self._chk(self.lib.lh2_core_set_tile(self.h, int(y0), int(y1)))

    def set_tile_bands(self, rank: int, nranks: int, band: int) -> None:
        self._chk(self.lib.lh2_core_set_tile_bands(self.h, int(rank), int(nranks), int(band)))

    def sync(self) -> None:
        self._chk(self.lib.lh2_core_sync(self.h))

    def accumulator(self) -> np.ndarray:
        out = np.zeros((self.h_, self.w, 4), np.float32)
        self._chk(self.lib.lh2_core_get_accumulator(self.h, _fp(out)))
        return out

    def frame(self) -> np.ndarray:
        out = np.zeros((self.h_, self.w, 4), np.float32)
        self._chk(self.lib.lh2_core_get_frame(self.h, _fp(out)))
        return out

    def copy_accumulator_rows(self, device_ptr: int, y0: int, y1: int) -> None:
        self._chk(self.lib.lh2_core_copy_accumulator_rows(self.h, C.c_void_p(device_ptr), int(y0), int(y1)))

    def pack_tile(self, device_ptr: int, order_torch: bool = True) -> None:
        """Pack the owned accumulator rows into device memory (asynchronously, on the core stream).
        With order_torch, torch's current stream is made to wait for it (no host synchronisation), so
        torch ops and collectives on the tile see the finished rows."""
        if order_torch:
            # the previous frame's gather may still read this tile on torch's / RCCL's stream: the core
            # stream waits for it (GPU-side wait, so that gather overlaps this frame's rendering), and
            # torch's stream for the pack (the pack launch's own stop event: no marker between kernels)
            import torch
            s = torch.cuda.current_stream().cuda_stream
            self._chk(self.lib.lh2_core_pack_tile_ordered(self.h, C.c_void_p(device_ptr), C.c_void_p(s)))
        else:
            self._chk(self.lib.lh2_core_pack_tile(self.h, C.c_void_p(device_ptr)))

    def copy_frame_async(self, device_ptr: int) -> None:
        """The last finalized frame into device memory, asynchronously on the core stream (the headless
        counterpart of the display copy: no host synchronisation)."""
        self._chk(self.lib.lh2_core_copy_frame_async(self.h, C.c_void_p(device_ptr)))

    def stream_ptr(self) -> int:
        s = C.c_void_p()
        self._chk(self.lib.lh2_core_stream(self.h, C.byref(s)))
        return s.value or 0

    def tile_rows(self) -> int:
        r = C.c_int(0)
        self._chk(self.lib.lh2_core_tile_rows(self.h, C.byref(r)))
        return r.value

    def ray_counts(self) -> np.ndarray:
        out = np.zeros(17, np.uint32)
        self._chk(self.lib.lh2_core_ray_counts(self.h, _up(out)))
        return out

    def trace_closest(self, org_tmin: np.ndarray, dir_tmax: np.ndarray) -> np.ndarray:
        o = np.ascontiguousarray(org_tmin, np.float32)
        d = np.ascontiguousarray(dir_tmax, np.float32)
        n = len(o)
        hits = np.zeros((n, 4), np.uint32)
        self._chk(self.lib.lh2_core_trace_closest(self.h, _fp(o), _fp(d), n, _up(hits)))
        return hits

    def trace_any(self, org_tmin: np.ndarray, dir_tmax: np.ndarray) -> np.ndarray:
        o = np.ascontiguousarray(org_tmin, np.float32)
        d = np.ascontiguousarray(dir_tmax, np.float32)
        n = len(o)
        mask = np.zeros((n + 31) // 32, np.uint32)
        self._chk(self.lib.lh2_core_trace_any(self.h, _fp(o), _fp(d), n, _up(mask)))
        return mask

    def trace_closest_device(self, ray_o_ptr: int, ray_d_ptr: int, n: int, hits_ptr: int, iterations: int = 1) -> float:
        ms = C.c_float(0)
        self._chk(self.lib.lh2_core_trace_closest_device(self.h, C.c_void_p(ray_o_ptr), C.c_void_p(ray_d_ptr), int(n),
                                                         C.c_void_p(hits_ptr), int(iterations), C.byref(ms)))
        return ms.value

    def generate_eye_rays(self, view: abi.ViewPyramid, R0: int, pass_: int):
        n = self.w * self.h_ * self.spp
        o = np.zeros((n, 4), np.float32)
        d = np.zeros((n, 4), np.float32)
        s = np.zeros((n, 8), np.float32)
        self._chk(self.lib.lh2_core_generate_eye_rays(self.h, C.byref(view), R0 & 0xffffffff, int(pass_), _fp(o), _fp(d),
                                                      _fp(s)))
        return o, d, s

    def debug_shadow_rays(self, cap: int):
        """Diagnostics: the last frame's queued shadow rays (O4, D4, potentials; potential.w holds the pixel
        index bits)."""
        o, d, p = (np.zeros((cap, 4), np.float32) for _ in range(3))
        n = C.c_int(0)
        self._chk(self.lib.lh2_core_debug_shadow_rays(self.h, _fp(o), _fp(d), _fp(p), int(cap), C.byref(n)))
        return o[:n.value], d[:n.value], p[:n.value]

    def debug_bvh4(self, cap: int | None = None):
        """Diagnostics: the scene's BVH4 nodes, (n, 32) float32 (f32 layout) and (n, 16) uint32 (quantized).
        Without cap the arrays are sized by a count-only call first (cap 0 returns the node count)."""
        n = C.c_int(0)
        if cap is None:
            self._chk(self.lib.lh2_core_debug_bvh4(self.h, None, None, 0, C.byref(n)))
            cap = n.value
        f = np.zeros((max(cap, 1), 32), np.float32)
        q = np.zeros((max(cap, 1), 16), np.uint32)
        self._chk(self.lib.lh2_core_debug_bvh4(self.h, _fp(f), q.ctypes.data, int(cap), C.byref(n)))
        return f[:n.value], q[:n.value]

    def debug_poison_tlas(self, value: float) -> None:
        """Test hook: fill both TLAS slots' node regions with `value` (stale memory behind a TLAS update's nodes)."""
        self._chk(self.lib.lh2_core_debug_poison_tlas(self.h, float(value)))

    def scene_info(self) -> dict:
        v = [C.c_int(0) for _ in range(4)]
        self._chk(self.lib.lh2_core_scene_info(self.h, *[C.byref(x) for x in v]))
        return dict(nodes=v[0].value, tris=v[1].value, max_depth=v[2].value, instances=v[3].value)


def xorshift_floats_native(seed: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.float32)
    load_library().lh2_xorshift_floats(seed & 0xffffffff, _fp(out), n)
    return out
