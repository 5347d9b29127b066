"""Record the CoreAPI call stream a RenderSystem would make, to replay it through the C++ vtable.

`CallRecorder` has the same methods as `core.RenderCore` / `oracle.Oracle` (so `Scene.load_into`
and `Scene.render_frame` drive it unchanged) and writes every call as a record
    u32 opcode, u32 payload bytes, payload
to a file.  `tools/headless_rendersystem.cpp` replays the file against libRenderCore_MI355X.so
through dlopen + dlsym("CreateCore") + the CoreAPI_Base vtable, exactly the way
RenderSystem/core_api_base.cpp:97-132 and rendersystem.cpp:22-301 reach a core, with no Python
and no flat C layer in between.  Payloads are the reference's own POD layouts (lh2_core_types.h).
"""
from __future__ import annotations

import ctypes as C
import struct

import numpy as np

from . import abi

OP = dict(SET_SKY=1, SET_MATERIALS=2, SET_GEOMETRY=3, SET_INSTANCE=4, UPDATE_TOPLEVEL=5, SET_LIGHTS=6,
          SETTING=7, SET_TARGET=8, RENDER=9, SET_PROBE=10, SET_TEXTURES=11)


class CallRecorder:
    def __init__(self, path):
        self.f = open(path, "wb")

    def close(self):
        if self.f:
            self.f.close()
            self.f = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _rec(self, op: str, payload: bytes) -> None:
        self.f.write(struct.pack("<II", OP[op], len(payload)))
        self.f.write(payload)

    # CoreAPI_Base-shaped methods (core_api_base.h:84-113) ------------------------------------
    def set_target(self, w, h, spp=1):
        self._rec("SET_TARGET", struct.pack("<III", w, h, spp))

    def setting(self, name, value):
        self._rec("SETTING", name.encode().ljust(32, b"\0")[:32] + struct.pack("<f", float(value)))

    def set_probe(self, x, y):
        self._rec("SET_PROBE", struct.pack("<ii", x, y))

    def set_textures(self, textures):
        """SetTextures( const CoreTexDesc*, int ) (core_api_base.h:100): per texture the descriptor's fields
        (width, height, flags, pixelCount, MIPlevels, storage) and its texels; the replay host points the
        descriptor at its copy of them (the core copies them during the call, rendercore.cpp:276-347)."""
        out = [struct.pack("<i", len(textures))]
        for t in textures:
            px = np.ascontiguousarray(t.pixels)
            d = t.desc(px)
            out.append(struct.pack("<IIIIIiI", d.width, d.height, d.flags, d.pixelCount, d.MIPlevels, d.storage, px.nbytes))
            out.append(px.tobytes())
        self._rec("SET_TEXTURES", b"".join(out))

    def set_materials(self, mats):
        arr = abi.material_array(mats)
        self._rec("SET_MATERIALS", struct.pack("<i", len(mats)) + bytes(arr))

    def set_lights(self, area=(), point=(), spot=(), directional=()):
        head = struct.pack("<iiii", len(area), len(point), len(spot), len(directional))
        body = b"".join(bytes(x) for group in (area, point, spot, directional) for x in group)
        self._rec("SET_LIGHTS", head + body)

    def set_sky(self, rgb):
        rgb = np.ascontiguousarray(rgb, np.float32)
        self._rec("SET_SKY", struct.pack("<II", rgb.shape[1], rgb.shape[0]) + rgb.tobytes())

    def set_geometry(self, idx, tris):
        tris = np.ascontiguousarray(tris, np.float32)
        n = len(tris)
        verts = np.zeros((3 * n, 4), np.float32)
        verts[0::3, :3] = tris[:, 32:35]
        verts[1::3, :3] = tris[:, 36:39]
        verts[2::3, :3] = tris[:, 40:43]
        verts[:, 3] = 1
        self._rec("SET_GEOMETRY", struct.pack("<ii", idx, n) + verts.tobytes() + tris.tobytes())

    def set_instance(self, idx, mesh, T=None):
        m = np.ascontiguousarray(np.eye(4, dtype=np.float32) if T is None else T, np.float32)
        self._rec("SET_INSTANCE", struct.pack("<ii", idx, mesh) + m.tobytes())

    def update_toplevel(self):
        self._rec("UPDATE_TOPLEVEL", b"")

    def render(self, view, converge=1):
        assert C.sizeof(view) == 68
        self._rec("RENDER", bytes(view) + struct.pack("<i", int(converge)))
