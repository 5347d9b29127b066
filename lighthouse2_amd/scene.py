"""Synthetic scenes for the benchmark configurations (BASELINE.json `configs`) and a
headless stand-in for the reference RenderSystem's call sequence.

The reference drives a core through RenderSystem::SynchronizeSceneData (rendersystem.cpp:214-222):
sky -> textures -> materials -> meshes (SetGeometry) -> instances + UpdateToplevel -> lights, then
per frame Setting("epsilon"), Setting("clampValue") and Render (rendersystem.cpp:228-238).
`Scene.load_into` and `Scene.render_frame` replay exactly that order on any object with the
CoreAPI method names (the MI355X core, or the CPU oracle in tests).
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

from . import abi

# ---------------------------------------------------------------------------------------------
# Marsaglia xorshift32 stream (platform/system.cpp:44-46), vectorised by GF(2) jump-ahead
# ---------------------------------------------------------------------------------------------
_MASK = 0xFFFFFFFF


def _step(s: int) -> int:
    s ^= (s << 13) & _MASK
    s ^= s >> 17
    s ^= (s << 5) & _MASK
    return s


def _apply(cols: list[int], v: int) -> int:
    r = 0
    j = 0
    while v:
        if v & 1:
            r ^= cols[j]
        v >>= 1
        j += 1
    return r


_JUMP_CACHE: dict[int, np.ndarray] = {}


def _jump_tables(log2b: int) -> np.ndarray:
    """Byte tables of M^(2^log2b) where M is the xorshift32 step as a GF(2) linear map."""
    if log2b in _JUMP_CACHE:
        return _JUMP_CACHE[log2b]
    cols = [_step(1 << j) for j in range(32)]
    for _ in range(log2b):
        cols = [_apply(cols, c) for c in cols]
    tab = np.zeros((4, 256), np.uint32)
    for k in range(4):
        for b in range(256):
            tab[k, b] = _apply(cols, b << (8 * k))
    _JUMP_CACHE[log2b] = tab
    return tab


def xorshift_uints(seed: int, n: int, log2b: int = 14) -> np.ndarray:
    """The first n values of RandomUInt() starting from `seed` (each value is the state after a step)."""
    B = 1 << log2b
    out = np.empty(n, np.uint32)
    s = seed & _MASK
    first = min(n, B)
    if log2b > 6 and first > 64:
        out[:first] = xorshift_uints(seed, first, 6)   # the first block by jumps of 64 (a Python loop of 64 steps)
    else:
        for i in range(first):
            s = _step(s)
            out[i] = s
    if n <= B:
        return out
    tab = _jump_tables(log2b)
    prev = out[:B].copy()
    pos = B
    while pos < n:
        nxt = tab[0][prev & 255] ^ tab[1][(prev >> 8) & 255] ^ tab[2][(prev >> 16) & 255] ^ tab[3][prev >> 24]
        m = min(B, n - pos)
        out[pos:pos + m] = nxt[:m]
        prev = nxt
        pos += m
    return out


def xorshift_floats(seed: int, n: int) -> np.ndarray:
    """RandomFloat() stream: RandomUInt() * 2.3283064365387e-10f in fp32 (platform/system.cpp:46)."""
    return xorshift_uints(seed, n).astype(np.float32) * np.float32(2.3283064365387e-10)


# ---------------------------------------------------------------------------------------------
# camera -> ViewPyramid (RenderSystem/camera.cpp:38-55 CalculateMatrix, :96-117 GetView)
# ---------------------------------------------------------------------------------------------
def _f3(*v) -> np.ndarray:
    return np.array(v, np.float32)


def _norm(v: np.ndarray) -> np.ndarray:
    return (v * (np.float32(1) / np.sqrt(np.float32(np.dot(v, v))))).astype(np.float32)


_LIBM = None


def _tanf(x: np.float32) -> np.float32:
    """C tanf (the reference's camera.cpp calls it on a float): libm through ctypes, so the screen size
    rounds exactly as Camera::GetView's does."""
    global _LIBM
    import ctypes
    if _LIBM is None:
        _LIBM = ctypes.CDLL("libm.so.6")
        _LIBM.tanf.restype = ctypes.c_float
        _LIBM.tanf.argtypes = [ctypes.c_float]
    return np.float32(_LIBM.tanf(float(x)))


def camera_view(pos, direction, fov_deg: float = 40.0, aspect: float = 16 / 9, focal: float = 5.0,
                aperture: float = 0.0, distortion: float = 0.0, pixel_height: int = 1080) -> abi.ViewPyramid:
    """Camera::GetView (RenderSystem/camera.cpp:96-117, CalculateMatrix :40-58) in float32, in the
    reference's evaluation order (helper_math.h host forms: normalize = v * (1 / sqrtf(dot)), length =
    sqrtf(dot), cross / dot component-wise); pinned bit for bit to the reference compiled from its
    sources (tests/test_golden.py::test_camera_view_matches_reference).  `direction` is used as given
    (Camera::direction is kept normalised by the app)."""
    f32 = np.float32

    def v3(x, y, z):
        return (f32(x), f32(y), f32(z))

    def add(a, b):
        return (f32(a[0] + b[0]), f32(a[1] + b[1]), f32(a[2] + b[2]))

    def sub(a, b):
        return (f32(a[0] - b[0]), f32(a[1] - b[1]), f32(a[2] - b[2]))

    def smul(s, a):                    # float * float3
        return (f32(s * a[0]), f32(s * a[1]), f32(s * a[2]))

    def vmul(a, s):                    # float3 * float
        return (f32(a[0] * s), f32(a[1] * s), f32(a[2] * s))

    def dot(a, b):
        return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))

    def cross(a, b):
        return (f32(f32(a[1] * b[2]) - f32(a[2] * b[1])), f32(f32(a[2] * b[0]) - f32(a[0] * b[2])),
                f32(f32(a[0] * b[1]) - f32(a[1] * b[0])))

    def normalize(a):
        return vmul(a, f32(f32(1) / np.sqrt(dot(a, a))))

    def length(a):
        return np.sqrt(dot(a, a))

    P = v3(*pos)
    z = v3(*direction)
    if abs(float(z[1])) > 0.99:
        y = v3(1, 0, 0)
    else:
        y = v3(0, 1, 0)
    x = normalize(cross(z, y))
    y = cross(x, z)
    right, up, forward = x, y, z
    fov, a, fd = f32(fov_deg), f32(aspect), f32(focal)
    pi = f32(3.14159265358979323846264)
    screen = _tanf(f32(f32(fov / f32(2)) / f32(f32(180) / pi)))
    C = add(P, smul(fd, forward))
    t_r = vmul(vmul(smul(screen, right), fd), a)          # screenSize * right * focalDistance * aspectRatio
    t_u = smul(f32(screen * fd), up)                        # screenSize * focalDistance * up
    p1 = add(sub(C, t_r), t_u)
    p2 = add(add(C, t_r), t_u)
    p3 = sub(sub(C, t_r), t_u)
    v = abi.ViewPyramid()
    v.pos = abi.float3(*map(float, P))
    v.p1 = abi.float3(*map(float, p1))
    v.p2 = abi.float3(*map(float, p2))
    v.p3 = abi.float3(*map(float, p3))
    v.aperture = float(f32(aperture))
    v.spreadAngle = float(f32(f32(f32(fov * pi) / f32(180)) / f32(pixel_height)))
    v.focalDistance = float(fd)
    v.distortion = float(f32(distortion))
    u_r = vmul(smul(screen, right), a)                      # screenSize * right * aspectRatio
    u_u = smul(screen, up)
    u1 = add(sub(C, u_r), u_u)
    u2 = add(add(C, u_r), u_u)
    u3 = sub(sub(C, u_r), u_u)
    v.imagePlane = float(f32(length(sub(u1, u2)) * length(sub(u1, u3))))
    return v


# ---------------------------------------------------------------------------------------------
# scene container + RenderSystem call order
# ---------------------------------------------------------------------------------------------
@dataclasses.dataclass
class Scene:
    meshes: list                       # CoreTri arrays (N, 44) float32
    instances: list                    # (mesh index, 4x4 row-major float32)
    materials: list                    # abi.CoreMaterial
    area_lights: list = dataclasses.field(default_factory=list)
    point_lights: list = dataclasses.field(default_factory=list)
    spot_lights: list = dataclasses.field(default_factory=list)
    dir_lights: list = dataclasses.field(default_factory=list)
    sky: np.ndarray | None = None      # (h, w, 3) float32
    textures: list = dataclasses.field(default_factory=list)   # Texture
    view: abi.ViewPyramid | None = None
    name: str = "scene"

    @property
    def tri_count(self) -> int:
        return int(sum(len(m) for m in self.meshes))

    def load_into(self, core) -> None:
        """RenderSystem::SynchronizeSceneData order (rendersystem.cpp:214-222)."""
        if self.sky is not None:
            core.set_sky(self.sky)
        if self.textures:
            core.set_textures(self.textures)
        core.set_materials(self.materials)
        if hasattr(core, "set_geometries"):      # the CPU oracle builds its meshes' BVHs in parallel
            core.set_geometries(self.meshes)
        else:
            for i, m in enumerate(self.meshes):
                core.set_geometry(i, m)
        for i, (mesh, T) in enumerate(self.instances):
            core.set_instance(i, mesh, T)
        core.set_instance(len(self.instances), -1, None)
        core.update_toplevel()
        core.set_lights(self.area_lights, self.point_lights, self.spot_lights, self.dir_lights)

    def render_frame(self, core, converge: int = 1, view: abi.ViewPyramid | None = None,
                     epsilon: float = 1e-4, clamp: float = 10.0) -> None:
        """RenderSystem::Render (rendersystem.cpp:228-238)."""
        core.setting("epsilon", epsilon)
        core.setting("clampValue", clamp)
        core.render(view or self.view, converge)


def tiled_order(w: int, h: int) -> np.ndarray:
    """Pixel index held by each ray slot when the core stores primary rays in 8x8 pixel blocks per wave
    (setting "tiledRays", k_camera): frame-order arrays indexed with this give the in-frame ray order."""
    r = np.arange(w * h, dtype=np.int64)
    x, y = r % w, r // w
    if w % 8 == 0:
        rb = r // (8 * w)
        full = rb < h // 8
        q = r - rb * 8 * w
        k = q & 63
        x = np.where(full, (q >> 6) * 8 + (k & 7), x)
        y = np.where(full, rb * 8 + (k >> 3), y)
    return y * w + x


def light_from_tri(tri: np.ndarray, tri_idx: int, inst_idx: int, radiance) -> abi.CoreLightTri:
    """HostAreaLight constructor + ConvertToCoreLightTri (host_light.cpp:25-62)."""
    v0 = tri[32:35].astype(np.float32)
    v1 = tri[36:39].astype(np.float32)
    v2 = tri[40:43].astype(np.float32)
    L = abi.CoreLightTri()
    c = (np.float32(0.333333) * (v0 + v1 + v2)).astype(np.float32)
    a = np.float32(np.linalg.norm(v1 - v0))
    b = np.float32(np.linalg.norm(v2 - v1))
    cc = np.float32(np.linalg.norm(v0 - v2))
    s = (a + b + cc) * np.float32(0.5)
    area = np.float32(math.sqrt(max(float(s * (s - a) * (s - b) * (s - cc)), 0.0)))
    rad = np.array(radiance, np.float32)
    E = rad * area
    L.centre = abi.float3(*map(float, c))
    L.N = abi.float3(float(tri[11]), float(tri[15]), float(tri[19]))
    L.area = float(area)
    L.radiance = abi.float3(*map(float, rad))
    L.energy = float(E[0] + E[1] + E[2])
    L.vertex0 = abi.float3(*map(float, v0))
    L.vertex1 = abi.float3(*map(float, v1))
    L.vertex2 = abi.float3(*map(float, v2))
    L.triIdx = tri_idx
    L.instIdx = inst_idx
    return L


def point_light(pos, radiance, energy: float | None = None) -> abi.CorePointLight:
    """HostScene::AddPointLight + HostPointLight::ConvertToCorePointLight (host_scene.cpp:568-577, host_light.cpp:68-75).
    RenderSystem never sets HostPointLight::energy (default 0, host_light.h:61), so a point light reaching the core through
    an unchanged RenderSystem has energy 0: its NEE potential (lights_shared.h:64-72) is 0 and it is never picked.
    energy=None keeps that; a number is what a direct user of the core ABI may store."""
    L = abi.CorePointLight()
    L.position = abi.float3(*map(float, pos))
    L.radiance = abi.float3(*map(float, radiance))
    L.energy = 0.0 if energy is None else float(energy)
    return L


def spot_light(pos, direction, cos_inner: float, cos_outer: float, radiance) -> abi.CoreSpotLight:
    """HostScene::AddSpotLight + ConvertToCoreSpotLight (host_scene.cpp:583-595, host_light.cpp:81-90): the direction as
    given (RenderSystem does not normalise it), the cone as cosines; the potential uses the radiance sum
    (lights_shared.h:78-95), so spot lights are sampled through an unchanged RenderSystem."""
    L = abi.CoreSpotLight()
    L.position = abi.float3(*map(float, pos))
    L.direction = abi.float3(*map(float, direction))
    L.radiance = abi.float3(*map(float, radiance))
    L.cosInner, L.cosOuter = float(cos_inner), float(cos_outer)
    return L


def directional_light(direction, radiance, energy: float | None = None) -> abi.CoreDirectionalLight:
    """HostScene::AddDirectionalLight + ConvertToCoreDirectionalLight (host_scene.cpp:601-610, host_light.cpp:96-102):
    the direction as given; energy, as for point lights, stays 0 through RenderSystem (None) unless set."""
    L = abi.CoreDirectionalLight()
    L.direction = abi.float3(*map(float, direction))
    L.radiance = abi.float3(*map(float, radiance))
    L.energy = 0.0 if energy is None else float(energy)
    return L


def quad_tris(N, pos, width: float, height: float, material: int) -> np.ndarray:
    """HostScene::AddQuad (host_scene.cpp:346-393): two triangles, explicit normal N."""
    N = _norm(_f3(*N))
    pos = _f3(*pos)
    tmp = _f3(0, 1, 0) if N[0] > 0.9 else _f3(1, 0, 0)
    T = (np.float32(0.5 * width) * _norm(np.cross(N, tmp).astype(np.float32))).astype(np.float32)
    B = (np.float32(0.5 * height) * _norm(np.cross(_norm(T), N).astype(np.float32))).astype(np.float32)
    v = [pos - B - T, pos + B - T, pos - B + T, pos + B - T, pos + B + T, pos - B + T]
    t = abi.new_tris(2)
    for k, (a, b, c) in enumerate(((v[0], v[1], v[2]), (v[3], v[4], v[5]))):
        for key in ("vN0", "vN1", "vN2"):
            t[k, abi.TRI[key]:abi.TRI[key] + 3] = N
        t[k, abi.TRI["Nx"]], t[k, abi.TRI["Ny"]], t[k, abi.TRI["Nz"]] = N
        t[k, 32:35], t[k, 36:39], t[k, 40:43] = a, b, c
        t.view(np.uint32)[k, abi.TRI["material"]] = material
        Tt = _norm((b - a).astype(np.float32))
        t[k, abi.TRI["T"]:abi.TRI["T"] + 3] = Tt
        t[k, abi.TRI["B"]:abi.TRI["B"] + 3] = _norm(np.cross(N, Tt).astype(np.float32))
        la, lb, lc = (np.linalg.norm(b - a), np.linalg.norm(c - b), np.linalg.norm(a - c))
        s = (la + lb + lc) * 0.5
        t[k, abi.TRI["area"]] = math.sqrt(max(s * (s - la) * (s - lb) * (s - lc), 0))
    return t


# ---------------------------------------------------------------------------------------------
# config 2: 100k random triangles
# ---------------------------------------------------------------------------------------------
def random_triangles(n: int = 100_000, seed: int = 0x12345678, edge: float = 0.5, spread: float = 10.0) -> np.ndarray:
    r = xorshift_floats(seed, 9 * n).reshape(n, 9)
    half = np.float32(spread / 2)
    v0 = r[:, 0:3] * np.float32(spread) - half
    e = np.float32(edge)
    v1 = v0 + (r[:, 3:6] - np.float32(0.5)) * e
    v2 = v0 + (r[:, 6:9] - np.float32(0.5)) * e
    return abi.tris_from_vertices(v0, v1, v2, 0)


def config2_scene(n: int = 100_000, width: int = 1920, height: int = 1080, sky: bool = False,
                  light: bool = False) -> Scene:
    """Primary-ray BVH2 config: xorshift32 seed 0x12345678, v0 ~ U[-5,5]^3, edges 0.5, camera (0,0,-12)
    looking +z, FOV 40, 16:9, aperture 0, distortion 0, focal distance 5; material 0 = white 0.8,
    roughness 1.  `sky` / `light` add an environment / an area light for parity runs."""
    tris = random_triangles(n)
    mats = [abi.make_material((0.8, 0.8, 0.8), roughness=1.0)]
    sc = Scene(meshes=[tris], instances=[(0, np.eye(4, dtype=np.float32))], materials=mats, name=f"config2-{n}")
    if light:
        mats.append(abi.make_material((20.0, 20.0, 18.0)))
        q = quad_tris((0, -1, 0), (0, 7.5, 0), 6, 6, 1)
        sc.meshes.append(q)
        q.view(np.int32)[:, abi.TRI["ltriIdx"]] = [0, 1]
        sc.instances.append((1, np.eye(4, dtype=np.float32)))
        sc.area_lights = [light_from_tri(q[i], i, 1, (20.0, 20.0, 18.0)) for i in range(2)]
    if sky:
        sc.sky = gradient_sky(64, 32)
    sc.view = camera_view((0, 0, -12), (0, 0, 1), fov_deg=40, aspect=width / height, focal=5, pixel_height=height)
    return sc


def gradient_sky(w: int = 64, h: int = 32) -> np.ndarray:
    y = np.linspace(1.0, 0.1, h, dtype=np.float32)[:, None]
    x = np.linspace(0.0, 1.0, w, dtype=np.float32)[None, :]
    ones = np.ones((h, w), np.float32)
    sky = np.stack([(0.4 * y + 0.1 * x) * ones, (0.5 * y + 0.05) * ones, (0.9 * y + 0.05 * (1 - x)) * ones], -1).astype(np.float32)
    return np.ascontiguousarray(sky)


# ---------------------------------------------------------------------------------------------
# config 3: procedural "Sponza-class" room
# ---------------------------------------------------------------------------------------------
def _grid_quads(origin, du, dv, nu: int, nv: int) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    o = np.asarray(origin, np.float32)
    du = np.asarray(du, np.float32)
    dv = np.asarray(dv, np.float32)
    i, j = np.meshgrid(np.arange(nu, dtype=np.float32), np.arange(nv, dtype=np.float32), indexing="ij")
    i = i.ravel()[:, None]
    j = j.ravel()[:, None]
    a = o + (i / nu) * du + (j / nv) * dv
    b = o + ((i + 1) / nu) * du + (j / nv) * dv
    c = o + ((i + 1) / nu) * du + ((j + 1) / nv) * dv
    d = o + (i / nu) * du + ((j + 1) / nv) * dv
    v0 = np.concatenate([a, a]).astype(np.float32)
    v1 = np.concatenate([b, c]).astype(np.float32)
    v2 = np.concatenate([c, d]).astype(np.float32)
    return v0, v1, v2


def _box(lo, hi, nseg: int):
    lo = np.asarray(lo, np.float32)
    hi = np.asarray(hi, np.float32)
    d = hi - lo
    ex, ey, ez = np.array([d[0], 0, 0], np.float32), np.array([0, d[1], 0], np.float32), np.array([0, 0, d[2]], np.float32)
    faces = [(lo, ey, ex), (lo + ez, ex, ey), (lo, ez, ey), (lo + ex, ey, ez), (lo, ex, ez), (lo + ey, ez, ex)]
    parts = [_grid_quads(o, u, v, nseg, nseg) for o, u, v in faces]
    return tuple(np.concatenate([p[k] for p in parts]) for k in range(3))


def _sphere(center, radius: float, nu: int, nv: int):
    """UV sphere: (v0, v1, v2) corners and their analytic vertex normals (smooth shading)."""
    th = np.linspace(0.0, np.pi, nv + 1)
    ph = np.linspace(0.0, 2 * np.pi, nu + 1)
    P = np.stack([np.sin(th)[:, None] * np.cos(ph)[None], np.cos(th)[:, None] * np.ones_like(ph)[None],
                  np.sin(th)[:, None] * np.sin(ph)[None]], -1)             # (nv+1, nu+1, 3) unit normals
    a, b, c, d = P[:-1, :-1], P[:-1, 1:], P[1:, :-1], P[1:, 1:]
    n0 = np.concatenate([a.reshape(-1, 3), b.reshape(-1, 3)])
    n1 = np.concatenate([b.reshape(-1, 3), d.reshape(-1, 3)])
    n2 = np.concatenate([c.reshape(-1, 3), c.reshape(-1, 3)])
    keep = np.linalg.norm(np.cross(n1 - n0, n2 - n0), axis=1) > 1e-9      # drop the degenerate pole tris
    n0, n1, n2 = (x[keep].astype(np.float32) for x in (n0, n1, n2))
    ctr = np.asarray(center, np.float32)
    r = np.float32(radius)
    return n0 * r + ctr, n1 * r + ctr, n2 * r + ctr, (n0, n1, n2)


def room_scene(target_tris: int = 1_000_000, width: int = 1920, height: int = 1080, seed: int = 0x1234,
               sky: bool = True) -> Scene:
    """Closed room 40 x 16 x 24 (tessellated walls), 32 columns, 10 smooth-shaded spheres (vertex
    normals), seeded clutter, two emissive quads.  Materials: 70 % roughness-1 diffuse (NEE), 20 %
    default roughness 0 (specular chain), 10 % glass (transmission 1, eta 1.5); lights radiance 50."""
    rng = np.random.default_rng(seed)
    mats = [
        abi.make_material((0.75, 0.75, 0.72), roughness=1.0),   # 0 floor / ceiling
        abi.make_material((0.7, 0.35, 0.3), roughness=1.0),     # 1 walls red
        abi.make_material((0.3, 0.45, 0.7), roughness=1.0),     # 2 walls blue
        abi.make_material((0.8, 0.8, 0.8)),                     # 3 specular (default roughness 0)
        abi.make_material((0.95, 0.95, 0.95), transmission=1.0, eta=1.5, absorption=(0.1, 0.05, 0.02)),  # 4 glass
        abi.make_material((0.6, 0.6, 0.4), roughness=1.0, metallic=0.3, specular=0.5),  # 5 diffuse mixed
        abi.make_material((50.0, 50.0, 50.0)),                  # 6 light
    ]
    # budget: walls 40 %, columns 20 %, clutter 40 %
    wall_budget = int(target_tris * 0.4)
    W, H, D = 40.0, 16.0, 24.0
    area_tot = 2 * (W * H + W * D + H * D)
    cell = math.sqrt(area_tot * 2 / max(wall_budget, 12))
    def nseg(x):
        return max(1, int(round(x / cell)))
    x0, x1, y0, y1, z0, z1 = -W / 2, W / 2, 0.0, H, -D / 2, D / 2
    walls = [
        ((x0, y0, z0), (W, 0, 0), (0, 0, D), nseg(W), nseg(D), 0),      # floor (normal +y)
        ((x0, y1, z0), (0, 0, D), (W, 0, 0), nseg(D), nseg(W), 0),      # ceiling (normal -y)
        ((x0, y0, z0), (0, H, 0), (W, 0, 0), nseg(H), nseg(W), 1),      # back wall z0 (normal +z)
        ((x0, y0, z1), (W, 0, 0), (0, H, 0), nseg(W), nseg(H), 2),      # front wall z1
        ((x0, y0, z0), (0, 0, D), (0, H, 0), nseg(D), nseg(H), 2),      # left wall x0
        ((x1, y0, z0), (0, H, 0), (0, 0, D), nseg(H), nseg(D), 1),      # right wall x1
    ]
    V0, V1, V2, M = [], [], [], []
    for o, du, dv, nu, nv, mat in walls:
        a, b, c = _grid_quads(o, du, dv, nu, nv)
        V0.append(a), V1.append(b), V2.append(c), M.append(np.full(len(a), mat, np.uint32))
    # 32 columns: 2 rows of 16 boxes
    col_budget = int(target_tris * 0.2)
    ns_col = max(1, int(math.sqrt(col_budget / 32 / 12)))
    for k in range(32):
        x = -18 + (k % 16) * 2.4
        z = -6.0 if k < 16 else 6.0
        a, b, c = _box((x - 0.4, 0, z - 0.4), (x + 0.4, H, z + 0.4), ns_col)
        V0.append(a), V1.append(b), V2.append(c)
        mat = 3 if k % 5 == 0 else 5 if k % 3 == 0 else 0
        M.append(np.full(len(a), mat, np.uint32))
    # 10 smooth spheres (vertex normals: exercises the hit barycentrics in GetShadingData)
    sph_budget = int(target_tris * 0.05)
    nu = max(6, int(math.sqrt(sph_budget / 10 / 2 * 2)))
    S0, S1, S2, SN, SM = [], [], [], [[], [], []], []
    for k in range(10):
        ctr = (-15 + k * 3.3, 1.0 + 0.6 * (k % 3), -1.5 if k % 2 else 1.5)
        a, b, c, vn = _sphere(ctr, 0.8 + 0.1 * (k % 4), nu, max(3, nu // 2))
        S0.append(a), S1.append(b), S2.append(c), SM.append(np.full(len(a), (4, 3, 0, 5)[k % 4], np.uint32))
        for i in range(3):
            SN[i].append(vn[i])
    spheres = abi.tris_from_vertices(np.concatenate(S0), np.concatenate(S1), np.concatenate(S2), np.concatenate(SM),
                                     vertex_normals=tuple(np.concatenate(x) for x in SN))
    # clutter: random boxes on the floor
    clutter_budget = target_tris - sum(len(a) for a in V0) - len(spheres)
    ns_cl = 2
    per_box = 12 * ns_cl * ns_cl
    nboxes = max(1, clutter_budget // per_box)
    pos = rng.uniform((-19, 0, -11), (19, 6, 11), size=(nboxes, 3)).astype(np.float32)
    size = rng.uniform(0.1, 0.6, size=(nboxes, 3)).astype(np.float32)
    matsel = rng.choice([0, 1, 2, 5, 3, 4], size=nboxes, p=[0.3, 0.15, 0.15, 0.1, 0.2, 0.1])
    base_a, base_b, base_c = _box((0, 0, 0), (1, 1, 1), ns_cl)
    a = (base_a[None] * size[:, None] + pos[:, None]).reshape(-1, 3)
    b = (base_b[None] * size[:, None] + pos[:, None]).reshape(-1, 3)
    c = (base_c[None] * size[:, None] + pos[:, None]).reshape(-1, 3)
    V0.append(a.astype(np.float32)), V1.append(b.astype(np.float32)), V2.append(c.astype(np.float32))
    M.append(np.repeat(matsel.astype(np.uint32), per_box))
    tris = abi.tris_from_vertices(np.concatenate(V0), np.concatenate(V1), np.concatenate(V2), np.concatenate(M))
    tris = np.concatenate([tris, spheres])
    # two emissive quads just below the ceiling, facing down
    q1 = quad_tris((0, -1, 0), (-8, H - 0.05, 0), 4, 4, 6)
    q2 = quad_tris((0, -1, 0), (8, H - 0.05, 0), 4, 4, 6)
    base = len(tris)
    lights = np.concatenate([q1, q2])
    lights.view(np.int32)[:, abi.TRI["ltriIdx"]] = np.arange(4)
    tris = np.concatenate([tris, lights])
    area = [light_from_tri(tris[base + i], base + i, 0, (50.0, 50.0, 50.0)) for i in range(4)]
    sc = Scene(meshes=[tris], instances=[(0, np.eye(4, dtype=np.float32))], materials=mats, area_lights=area,
               name=f"room-{len(tris)}")
    if sky:
        sc.sky = gradient_sky(64, 32)
    sc.view = camera_view((0, 6, 11), (0, -0.15, -1), fov_deg=60, aspect=width / height, focal=5,
                          pixel_height=height)
    return sc


# ---------------------------------------------------------------------------------------------
# config 5: instanced meshes with per-frame transforms
# ---------------------------------------------------------------------------------------------
def rotation_y(a: float) -> np.ndarray:
    """mat4::RotateY (common_types.h:490)."""
    m = np.eye(4, dtype=np.float32)
    c, s = np.float32(math.cos(a)), np.float32(math.sin(a))
    m[0, 0], m[0, 2], m[2, 0], m[2, 2] = c, s, -s, c
    return m


def instanced_scene(meshes: int = 100, tris_per_mesh: int = 100_000, width: int = 1920, height: int = 1080,
                    grid: int = 10, spacing: float = 12.0) -> Scene:
    mlist = [random_triangles(tris_per_mesh, seed=0x12345678 + k) for k in range(meshes)]
    inst = []
    for k in range(meshes):
        T = np.eye(4, dtype=np.float32)
        T[0, 3] = (k % grid - (grid - 1) / 2) * spacing
        T[2, 3] = (k // grid - (grid - 1) / 2) * spacing
        inst.append((k, T))
    mats = [abi.make_material((0.8, 0.8, 0.8), roughness=1.0)]
    sc = Scene(meshes=mlist, instances=inst, materials=mats, name=f"instanced-{meshes}x{tris_per_mesh}")
    sc.sky = gradient_sky(64, 32)
    sc.view = camera_view((0, 60, -80), (0, -0.6, 1), fov_deg=50, aspect=width / height, pixel_height=height)
    return sc


def animate_instances(sc: Scene, frame: int, seed: int = 7) -> None:
    """Seeded per-frame rotations of every instance (the refit stress of config 5)."""
    rng = np.random.default_rng(seed + frame)
    angles = rng.uniform(0, 2 * math.pi, size=len(sc.instances))
    new = []
    for (mesh, T), a in zip(sc.instances, angles):
        R = rotation_y(float(a))
        M = R.copy()
        M[:, 3] = T[:, 3]
        new.append((mesh, M.astype(np.float32)))
    sc.instances = new


# ---------------------------------------------------------------------------------------------
# texture maps: HostTexture-equivalent texel preparation + a textured scene
# ---------------------------------------------------------------------------------------------
MIPLEVELCOUNT = 5          # common_settings.h:49
TEX_NORMALMAP, TEX_HDR = 2, 8   # HostTexture flags (host_texture.h:42-44)


def pixels_needed(w: int, h: int, levels: int) -> int:
    """HostTexture::PixelsNeeded (host_texture.cpp:117-122)."""
    n = 0
    for _ in range(levels):
        n += w * h
        w >>= 1
        h >>= 1
    return n


def construct_mipmaps(base: np.ndarray) -> np.ndarray:
    """HostTexture::ConstructMIPmaps (host_texture.cpp:128-151) on uint32 texels (h, w): each level
    averages 2x2 blocks of bytes 0..2 (>> 2 of the sum) and keeps the minimum of byte 3."""
    h, w = base.shape
    out = [base.reshape(-1).astype(np.uint32)]
    src = base.astype(np.uint32)
    for _ in range(1, MIPLEVELCOUNT):
        h2, w2 = src.shape[0] >> 1, src.shape[1] >> 1
        if h2 == 0 or w2 == 0:
            out.append(np.zeros(0, np.uint32))
            src = np.zeros((h2, w2), np.uint32)
            continue
        q = [src[0:2 * h2:2, 0:2 * w2:2], src[0:2 * h2:2, 1:2 * w2:2], src[1:2 * h2:2, 0:2 * w2:2], src[1:2 * h2:2, 1:2 * w2:2]]
        a = np.minimum(np.minimum(q[0] >> 24, q[1] >> 24), np.minimum(q[2] >> 24, q[3] >> 24))
        ch = [sum(((x >> s) & 255) for x in q) >> 2 for s in (16, 8, 0)]
        dst = (a << 24) + (ch[0] << 16) + (ch[1] << 8) + ch[2]
        out.append(dst.reshape(-1).astype(np.uint32))
        src = dst
    return np.concatenate(out).astype(np.uint32)


@dataclasses.dataclass
class Texture:
    """Texel data as RenderSystem hands it to the core (HostTexture::ConvertToCoreTexDesc,
    host_texture.cpp:43-67): LDR textures carry all MIPLEVELCOUNT levels; normal maps use NRM32."""
    pixels: np.ndarray        # uint32 texels, levels concatenated
    width: int
    height: int
    flags: int = 0
    storage: int = 0          # 0 ARGB32, 1 ARGB128, 2 NRM32
    mips: int = MIPLEVELCOUNT

    def desc(self, keep: np.ndarray) -> abi.CoreTexDesc:
        d = abi.CoreTexDesc()
        d.idata = keep.ctypes.data
        d.width, d.height, d.flags = self.width, self.height, self.flags
        d.pixelCount = int(keep.size if self.storage != 1 else keep.size // 4)
        d.firstPixel, d.MIPlevels, d.storage = 0, self.mips, self.storage
        return d


def make_texture(rgba: np.ndarray, normal_map: bool = False) -> Texture:
    """rgba: (h, w, 4) uint8, bytes in texel order (byte 0 = the texel's x component)."""
    rgba = np.ascontiguousarray(rgba, np.uint8)
    h, w = rgba.shape[:2]
    base = rgba.view(np.uint32).reshape(h, w)
    px = construct_mipmaps(base)
    assert px.size == pixels_needed(w, h, MIPLEVELCOUNT)
    return Texture(px, w, h, TEX_NORMALMAP if normal_map else 0, 2 if normal_map else 0)


def _tex_pattern(w: int, h: int, seed: int, kind: str) -> np.ndarray:
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    if kind == "checker":
        c = ((x // 8 + y // 8) % 2).astype(np.float32)
        rgb = np.stack([0.25 + 0.7 * c, 0.3 + 0.4 * c, 0.8 - 0.6 * c], -1)
        rgb = rgb + rng.uniform(-0.1, 0.1, rgb.shape)
        a = np.ones((h, w))
    elif kind == "detail":
        rgb = 0.5 + 0.2 * np.stack([np.sin(x * 0.7), np.cos(y * 0.9), np.sin((x + y) * 0.4)], -1)
        a = np.ones((h, w))
    elif kind == "cutout":
        rgb = np.stack([0.9 * np.ones((h, w)), 0.6 + 0.3 * (x / w), 0.2 + 0.5 * (y / h)], -1)
        a = (((x - w / 2) ** 2 + (y - h / 2) ** 2) > (0.3 * w) ** 2).astype(np.float32) * ((x // 4) % 3 != 0)
    elif kind == "gray":
        rgb = np.repeat((0.2 + 0.8 * rng.uniform(0, 1, (h, w, 1))), 3, -1)
        a = np.ones((h, w))
    else:  # normal map: tilted bumps, z up, mapped to [0, 1]
        nx = 0.5 * np.sin(x * 2 * np.pi / 16) + rng.uniform(-0.1, 0.1, (h, w))
        ny = 0.5 * np.cos(y * 2 * np.pi / 16)
        nz = np.sqrt(np.maximum(0.05, 1 - nx * nx - ny * ny))
        rgb = np.stack([nx, ny, nz], -1) * 0.5 + 0.5
        a = np.ones((h, w))
    px = np.concatenate([np.clip(rgb, 0, 1), a[..., None]], -1)
    return np.ascontiguousarray((px * 255.999).astype(np.uint8))


def _uv_tris(v0, v1, v2, uv0, uv1, uv2, material, vertex_normals=None, tex_area: float = 64 * 64) -> np.ndarray:
    """CoreTri records with texture coordinates, tangent frame and LOD: T / B from the UV gradient
    (HostMesh::BuildFromIndexedData convention), triLOD = 0.5 log2(texel area / triangle area)."""
    t = abi.tris_from_vertices(v0, v1, v2, material, vertex_normals=vertex_normals)
    uv0, uv1, uv2 = (np.asarray(a, np.float32) for a in (uv0, uv1, uv2))
    t[:, abi.TRI["u"]:abi.TRI["u"] + 3] = np.stack([uv0[:, 0], uv1[:, 0], uv2[:, 0]], 1)
    t[:, abi.TRI["v"]:abi.TRI["v"] + 3] = np.stack([uv0[:, 1], uv1[:, 1], uv2[:, 1]], 1)
    e1, e2 = (v1 - v0).astype(np.float32), (v2 - v0).astype(np.float32)
    d1, d2 = uv1 - uv0, uv2 - uv0
    det = d1[:, 0] * d2[:, 1] - d2[:, 0] * d1[:, 1]
    det = np.where(np.abs(det) < 1e-12, 1.0, det)[:, None]
    T = (e1 * d2[:, 1:2] - e2 * d1[:, 1:2]) / det
    B = (e2 * d1[:, 0:1] - e1 * d2[:, 0:1]) / det
    T = T / np.maximum(np.linalg.norm(T, axis=1, keepdims=True), 1e-12)
    B = B / np.maximum(np.linalg.norm(B, axis=1, keepdims=True), 1e-12)
    t[:, abi.TRI["T"]:abi.TRI["T"] + 3] = T
    t[:, abi.TRI["B"]:abi.TRI["B"] + 3] = B
    area = 0.5 * np.linalg.norm(np.cross(e1, e2), axis=1)
    tarea = 0.5 * np.abs(det[:, 0]) * tex_area
    t[:, abi.TRI["LOD"]] = (0.5 * np.log2(np.maximum(tarea, 1e-12) / np.maximum(area, 1e-12))).astype(np.float32)
    t[:, abi.TRI["alpha"]:abi.TRI["alpha"] + 3] = 0.0
    return t.astype(np.float32)


def _grid_uv(origin, du, dv, nu, nv, repeat):
    a, b, c = _grid_quads(origin, du, dv, nu, nv)
    o, du, dv = (np.asarray(x, np.float32) for x in (origin, du, dv))
    def uv(p):
        rel = p - o
        return np.stack([rel @ du / (du @ du), rel @ dv / (dv @ dv)], 1).astype(np.float32) * np.float32(repeat)
    return a, b, c, uv(a), uv(b), uv(c)


def textured_scene(width: int = 1920, height: int = 1080, tess: int = 24, instances: int = 2) -> Scene:
    """Every texture path of GetShadingData (material_shared.h:99-171): trilinear diffuse map + detail
    map, alpha cut-out, normal map + detail normal map (NRM32), roughness map, UV scale / offset;
    smooth sphere with a diffuse map; an area light; mesh instanced with rotations and scale."""
    tex = [make_texture(_tex_pattern(64, 64, 1, "checker")), make_texture(_tex_pattern(32, 32, 2, "detail")),
           make_texture(_tex_pattern(64, 64, 3, "gray")), make_texture(_tex_pattern(32, 32, 4, "normal"), normal_map=True),
           make_texture(_tex_pattern(16, 16, 5, "normal"), normal_map=True), make_texture(_tex_pattern(64, 64, 6, "cutout"))]
    def mat(color, tid=None, detail=None, nrm=None, nrm2=None, rough=None, alpha=False, uvs=(1, 1), uvo=(0, 0), **kw):
        m = abi.make_material(color, **kw)
        for field, t in (("color", tid), ("detailColor", detail), ("normals", nrm), ("detailNormals", nrm2)):
            if t is not None:
                f = getattr(m, field)
                f.textureID = t
                f.uvscale[0], f.uvscale[1] = uvs
                f.uvoffset[0], f.uvoffset[1] = uvo
        if rough is not None:
            m.roughness.textureID = rough
        if alpha:
            m.flags |= 2
        return m
    mats = [mat((0.9, 0.9, 0.9), tid=0, detail=1, rough=2, roughness=0.6, uvs=(1.5, 1.25), uvo=(0.25, 0.1)),   # 0 floor
            mat((0.8, 0.7, 0.6), tid=0, nrm=3, nrm2=4, roughness=1.0),                                          # 1 wall
            mat((1.0, 1.0, 1.0), tid=5, alpha=True, roughness=1.0),                                             # 2 cut-out
            abi.make_material((30.0, 30.0, 26.0)),                                                              # 3 light
            mat((0.9, 0.8, 0.7), tid=0, nrm=3, roughness=0.8, metallic=0.2, uvs=(4, 2)),                       # 4 sphere
            mat((0.7, 0.8, 0.9), tid=1, roughness=0.0)]                                                         # 5 specular textured
    parts = []
    a, b, c, ua, ub, uc = _grid_uv((-6, 0, -6), (12, 0, 0), (0, 0, 12), tess, tess, 3.0)
    parts.append(_uv_tris(a, b, c, ua, ub, uc, 0))
    a, b, c, ua, ub, uc = _grid_uv((-6, 0, 6), (12, 0, 0), (0, 8, 0), tess, tess // 2, 2.0)
    parts.append(_uv_tris(a, c, b, ua, uc, ub, 1))
    a, b, c, ua, ub, uc = _grid_uv((-2.5, 0.2, 1.5), (5, 0, 0), (0, 4, 0), 4, 4, 1.0)
    parts.append(_uv_tris(a, c, b, ua, uc, ub, 2))
    a, b, c, ua, ub, uc = _grid_uv((3.0, 0.2, -1.0), (0, 0, 3), (0, 3, 0), 3, 3, 1.0)
    parts.append(_uv_tris(a, c, b, ua, uc, ub, 5))
    s0, s1, s2, vn = _sphere((-3.0, 1.4, -1.0), 1.3, 2 * tess, tess)
    def suv(n):
        return np.stack([np.arctan2(n[:, 2], n[:, 0]) / (2 * np.pi) + 0.5, np.arccos(np.clip(n[:, 1], -1, 1)) / np.pi], 1)
    parts.append(_uv_tris(s0, s1, s2, suv(vn[0]), suv(vn[1]), suv(vn[2]), 4, vertex_normals=vn))
    tris = np.concatenate(parts).astype(np.float32)
    light = quad_tris((0, -1, 0), (0, 7.5, 0), 3, 3, 3)
    base = len(tris)
    light.view(np.int32)[:, abi.TRI["ltriIdx"]] = np.arange(2)
    tris = np.concatenate([tris, light])
    area = [light_from_tri(tris[base + i], base + i, 0, (30.0, 30.0, 26.0)) for i in range(2)]
    inst = [(0, np.eye(4, dtype=np.float32))]
    for k in range(1, instances):
        T = rotation_y(0.6 * k) * np.float32(0.5)
        T[3, 3] = 1
        T[:3, 3] = (14.0 * k, 0.0, 3.0)
        inst.append((0, T.astype(np.float32)))
    sc = Scene(meshes=[tris], instances=inst, materials=mats, area_lights=area, textures=tex, name="textured")
    sc.sky = gradient_sky(64, 32)
    sc.view = camera_view((2, 5, -12), (0.25, -0.3, 1), fov_deg=60, aspect=width / height, focal=5, pixel_height=height)
    return sc


def chord_order(O, D, lo, hi, cut, segs=8):
    """The order in which a frame's trace launch takes rays that a shade launch wrote into two-ended
    segments (RenderCore setting chordSplit, ShadeParams::chordCut): per segment (the launch's
    eighths), the rays whose chord through the scene box [lo, hi] exceeds cut x its largest extent,
    in order, then the others in reverse (they are written from the segment's end).  Returns the
    permutation."""
    lo, hi = np.asarray(lo, np.float64), np.asarray(hi, np.float64)
    c = cut * float((hi - lo).max())
    with np.errstate(divide="ignore", invalid="ignore"):
        t = np.minimum.reduce([np.maximum((lo[k] - O[:, k]) / D[:, k], (hi[k] - O[:, k]) / D[:, k]) for k in range(3)])
    n = len(O)
    seg = (n + segs - 1) // segs
    out = []
    for k in range(segs):
        idx = np.arange(k * seg, min(n, (k + 1) * seg))
        late = t[idx] <= c if cut > 0 else np.zeros(len(idx), bool)
        out += [idx[~late], idx[late][::-1]]
    return np.concatenate(out)


def mesh_box(tris):
    """The box of a mesh's vertices (CoreTri records)."""
    t = np.asarray(tris)
    v = np.concatenate([t[:, abi.TRI["vertex0"]:abi.TRI["vertex0"] + 3], t[:, abi.TRI["vertex1"]:abi.TRI["vertex1"] + 3],
                        t[:, abi.TRI["vertex2"]:abi.TRI["vertex2"] + 3]], 0)
    return v.min(0), v.max(0)


def bounce_rays(tris, O4, D4, hits, seed=1):
    """Diffuse 'bounce' rays from primary hits, as the first shade pass emits them (bench.py's roofline
    launch, tools/trace_kernel_bench.py, the bounce-visits fixture): cosine-weighted around the face
    normal of each hit (flipped toward the viewer), origin offset 1e-4 along it.  Misses are dropped
    (compacted, input order kept).  Returns O (tmin 0), D (tmax 1e34) as float32 [n, 4]."""
    hit = hits[:, 1] != 0xFFFFFFFF
    idx = np.nonzero(hit)[0]
    tri = hits[idx, 1].astype(np.int64)
    t = hits[idx, 0].view(np.float32)
    P = O4[idx, :3] + t[:, None] * D4[idx, :3]
    N = np.stack([tris[tri, abi.TRI["Nx"]], tris[tri, abi.TRI["Ny"]], tris[tri, abi.TRI["Nz"]]], 1)
    N = np.where(((N * D4[idx, :3]).sum(1) > 0)[:, None], -N, N)
    rng = np.random.default_rng(seed)
    r0, r1 = rng.random(len(idx)), rng.random(len(idx))
    phi = 2 * np.pi * r0
    local = np.stack([np.cos(phi) * np.sqrt(1 - r1), np.sin(phi) * np.sqrt(1 - r1), np.sqrt(r1)], 1)
    a = np.where(np.abs(N[:, 0:1]) > 0.9, np.array([[0, 1, 0]]), np.array([[1, 0, 0]]))
    T = np.cross(N, a)
    T /= np.linalg.norm(T, axis=1, keepdims=True)
    B = np.cross(N, T)
    d = local[:, 0:1] * T + local[:, 1:2] * B + local[:, 2:3] * N
    o = P + 1e-4 * N
    O = np.concatenate([o, np.zeros((len(o), 1))], 1).astype(np.float32)
    D = np.concatenate([d, np.full((len(d), 1), 1e34)], 1).astype(np.float32)
    return O, D


# ---------------------------------------------------------------------------------------------
# config 1: tinyapp's default scene (BASELINE.json configs[0], apps/tinyapp/main.cpp:34-45)
# ---------------------------------------------------------------------------------------------
TINYAPP_FIXTURE = __import__("pathlib").Path(__file__).resolve().parents[1] / "tests" / "golden" / "config1_tinyapp.npz"


def _normalize_rows(v: np.ndarray) -> np.ndarray:
    """helper_math.h normalize on the host: v * (1 / sqrtf(dot(v, v))), float32."""
    d = (v * v).sum(1, dtype=np.float32).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        return (v * (np.float32(1) / np.sqrt(d))[:, None]).astype(np.float32)


def _consistent_alpha(nnv: np.ndarray) -> np.ndarray:
    """The consistent-normal parameter per vertex: acosf(nnv) * (1 + 0.03632 (1 - nnv)^2) (host_mesh.cpp:190-196, 499-503)."""
    nnv = nnv.astype(np.float32)
    return (np.arccos(nnv).astype(np.float32) * (np.float32(1) + np.float32(0.03632) * (np.float32(1) - nnv) * (np.float32(1) - nnv))).astype(np.float32)


def _gltf_primitive_tris(P, Nv, U, ind, material: int) -> np.ndarray:
    """HostMesh::BuildFromIndexedData (host_mesh.cpp:477-569) for one glTF primitive with normals and uvs."""
    i0, i1, i2 = ind[0::3], ind[1::3], ind[2::3]
    v0, v1, v2 = P[i0], P[i1], P[i2]
    N = _normalize_rows(np.cross(v1 - v0, v2 - v0).astype(np.float32))
    vN0, vN1, vN2 = Nv[i0], Nv[i1], Nv[i2]
    d = lambda a, b: (a * b).sum(1, dtype=np.float32).astype(np.float32)
    flip = (d(N, vN0) < 0) & (d(N, vN1) < 0) & (d(N, vN2) < 0)
    Nf = np.where(flip[:, None], -N, N).astype(np.float32)        # flipped for the alphas only
    m0 = np.fmax(np.float32(0.7), d(vN0, Nf))   # fmaxf: a NaN dot (degenerate face) gives 0.7
    m1 = np.fmax(np.float32(0.7), d(vN1, Nf))
    m2 = np.fmax(np.float32(0.7), d(vN2, Nf))
    alpha = np.ones(len(P), np.float32)
    # sequential, with the reference's update of vertices 1 and 2 from vertex 0's value (host_mesh.cpp:497-499)
    for t in range(len(i0)):
        a0 = min(alpha[i0[t]], m0[t])
        alpha[i0[t]] = a0
        alpha[i1[t]] = min(a0, m1[t])
        alpha[i2[t]] = min(a0, m2[t])
    alpha = _consistent_alpha(alpha)
    t = abi.new_tris(len(i0))
    for k, vn in zip(("vN0", "vN1", "vN2"), (vN0, vN1, vN2)):
        t[:, abi.TRI[k]:abi.TRI[k] + 3] = vn
    t[:, abi.TRI["Nx"]], t[:, abi.TRI["Ny"]], t[:, abi.TRI["Nz"]] = N[:, 0], N[:, 1], N[:, 2]
    t[:, 32:35], t[:, 36:39], t[:, 40:43] = v0, v1, v2
    t[:, abi.TRI["alpha"]], t[:, abi.TRI["alpha"] + 1], t[:, abi.TRI["alpha"] + 2] = alpha[i0], alpha[i1], alpha[i2]
    uv0, uv1, uv2 = U[i0], U[i1], U[i2]
    # CoreTri u / v fields: (u0, u1, u2) at TRI["u"], (v0, v1, v2) at TRI["v"] (common_classes.h:126-154)
    t[:, abi.TRI["u"]:abi.TRI["u"] + 3] = np.stack([uv0[:, 0], uv1[:, 0], uv2[:, 0]], 1)
    t[:, abi.TRI["v"]:abi.TRI["v"] + 3] = np.stack([uv0[:, 1], uv1[:, 1], uv2[:, 1]], 1)
    uv01, uv02 = (uv1 - uv0).astype(np.float32), (uv2 - uv0).astype(np.float32)
    e1, e2 = (v1 - v0).astype(np.float32), (v2 - v0).astype(np.float32)
    edges = (d(uv01, uv01) == 0) | (d(uv02, uv02) == 0)
    T_e = _normalize_rows(e1)
    B_e = _normalize_rows(np.cross(N, T_e).astype(np.float32))
    T_u = _normalize_rows((e1 * uv02[:, 1:2] - e2 * uv01[:, 1:2]).astype(np.float32))
    B_u = _normalize_rows((e2 * uv01[:, 0:1] - e1 * uv02[:, 0:1]).astype(np.float32))
    t[:, abi.TRI["T"]:abi.TRI["T"] + 3] = np.where(edges[:, None], T_e, T_u)
    t[:, abi.TRI["B"]:abi.TRI["B"] + 3] = np.where(edges[:, None], B_e, B_u)
    t.view(np.uint32)[:, abi.TRI["material"]] = material
    return t


def _obj_tris(P, Nrm, fv, fn, fmat) -> np.ndarray:
    """HostMesh::LoadGeometryFromOBJ (host_mesh.cpp:131-305) for a smooth-shaded OBJ without texture coordinates."""
    v0, v1, v2 = P[fv[:, 0]], P[fv[:, 1]], P[fv[:, 2]]
    vN0, vN1, vN2 = Nrm[fn[:, 0]], Nrm[fn[:, 1]], Nrm[fn[:, 2]]
    d = lambda a, b: (a * b).sum(1, dtype=np.float32).astype(np.float32)
    # alphas per normal index: the face normal flipped when against all three vertex normals (:173-184)
    N0 = _normalize_rows(np.cross(v1 - v0, v2 - v0).astype(np.float32))
    flip = (d(N0, vN0) < 0) & (d(N0, vN1) < 0) & (d(N0, vN2) < 0)
    Na = np.where(flip[:, None], -N0, N0).astype(np.float32)
    alpha = np.ones(len(Nrm), np.float32)
    for k, vn in enumerate((vN0, vN1, vN2)):
        np.fmin.at(alpha, fn[:, k], np.fmax(np.float32(0.7), d(vn, Na)))
    alpha = _consistent_alpha(alpha)
    # the triangle records: face normal flipped when against vertex normal 0 (:253)
    e1, e2 = (v1 - v0).astype(np.float32), (v2 - v0).astype(np.float32)
    N = _normalize_rows(np.cross(e1, e2).astype(np.float32))
    N = np.where((d(N, vN0) < 0)[:, None], -N, N).astype(np.float32)
    t = abi.new_tris(len(fv))
    for k, vn in zip(("vN0", "vN1", "vN2"), (vN0, vN1, vN2)):
        t[:, abi.TRI[k]:abi.TRI[k] + 3] = vn
    t[:, abi.TRI["Nx"]], t[:, abi.TRI["Ny"]], t[:, abi.TRI["Nz"]] = N[:, 0], N[:, 1], N[:, 2]
    t[:, 32:35], t[:, 36:39], t[:, 40:43] = v0, v1, v2
    T = _normalize_rows(e1)
    t[:, abi.TRI["T"]:abi.TRI["T"] + 3] = T
    t[:, abi.TRI["B"]:abi.TRI["B"] + 3] = _normalize_rows(np.cross(N, T).astype(np.float32))
    t[:, abi.TRI["alpha"]], t[:, abi.TRI["alpha"] + 1], t[:, abi.TRI["alpha"] + 2] = alpha[fn[:, 0]], alpha[fn[:, 1]], alpha[fn[:, 2]]
    t.view(np.uint32)[:, abi.TRI["material"]] = fmat.astype(np.uint32)
    return t


# the stand-in for the one pica texture image missing from the reference (Wax_Pastel_Label_02_baseColor.png,
# .MISSING_LARGE_BLOBS): 512 x 512 texels of opaque white, so the material it colours (baseColorFactor 1) shades
# as it would untextured; every other texture is the reference's own image
MISSING_TEXTURE_RGBA = (512, 512, (255, 255, 255, 255))
TEX_LDR = 4                # HostTexture::LDR (host_texture.h:42)


def _gltf_texture(png: np.ndarray) -> Texture:
    """HostScene::AddScene's texture conversion (host_scene.cpp:260-271): the glTF image as tinygltf decodes it
    (stb_image, 8-bit RGBA with req_comp 4, first row first: tiny_gltf.h:2202-2286), memcpy'd into idata, flags
    LDR, MIP levels by ConstructMIPmaps (no FLIPPED / LINEARIZED mods on this path).  PNG is lossless, so PIL's
    decode (palette and transparency expanded to RGBA, like stb_image) gives the same bytes."""
    if png.size == 0:
        w, h, rgba = MISSING_TEXTURE_RGBA
        img = np.empty((h, w, 4), np.uint8)
        img[...] = np.array(rgba, np.uint8)
    else:
        import io
        from PIL import Image
        im = Image.open(io.BytesIO(png.tobytes()))
        assert im.mode in ("P", "RGB", "RGBA", "L", "LA"), im.mode   # 8 bits per channel
        img = np.asarray(im.convert("RGBA"), np.uint8)
    t = make_texture(img)
    t.flags = TEX_LDR
    return t


def tinyapp_scene(width: int = 640, height: int = 400, path=None) -> Scene:
    """tinyapp's PrepareScene (apps/tinyapp/main.cpp:34-45) from the committed fixture
    (tools/make_config1_fixture.py): the pica glTF diorama (170 meshes, one instance per node, the root node
    rotated by RotateX(-pi/2)), legocar.obj at scale 10 (placed as the main loop's first frame places it:
    Translate(0, 5, 0)), and the light quad (0, -1, 0) at (0, 26, 0), 6.9 x 6.9, radiance (100, 100, 80).
    Materials: glTF base colour / metallic / roughness factors and base colour textures (host_material.cpp:77-103;
    the six glTF textures as AddScene converts them, _gltf_texture, one a documented stand-in for the image missing
    from the reference), the .mtl Kd colours with tinyobjloader's default shininess (roughness 0), the
    light.  The camera is tinyapp's default (no camera.xml ships with the app: Camera's defaults, camera.h:33-44:
    at the origin looking down +z, FOV 40, focal distance 5, aperture EPSILON, distortion 0.05)."""
    f = np.load(path or TINYAPP_FIXTURE)
    meshes, materials = [], []
    # the glTF textures, in AddScene order (textureBase 0: the first scene loaded)
    textures = [_gltf_texture(f[f"pica_tex_png_{i}"]) for i in range(int(f["pica_tex_count"]))]
    for c, m, r, t in zip(f["pica_mat_color"], f["pica_mat_metallic"], f["pica_mat_roughness"], f["pica_mat_tex"]):
        mat = abi.make_material(tuple(float(x) for x in c), roughness=None if np.isnan(r) else float(r),
                                metallic=None if np.isnan(m) else float(m))
        if t >= 0:
            mat.color.textureID = int(t)      # baseColorTexture index + textureBase (host_material.cpp:95-98)
        materials.append(mat)
    prim_mesh, prim_mat, prim_v, prim_i = f["pica_prim_mesh"], f["pica_prim_mat"], f["pica_prim_v"], f["pica_prim_i"]
    P, Nv, U, I = f["pica_pos"], f["pica_nrm"], f["pica_uv"], f["pica_idx"]
    per_mesh = [[] for _ in range(int(f["pica_meshes"]))]
    for k in range(len(prim_mesh)):
        vb, vc = prim_v[k]
        ib, ic = prim_i[k]
        per_mesh[prim_mesh[k]].append(_gltf_primitive_tris(P[vb:vb + vc], Nv[vb:vb + vc], U[vb:vb + vc], I[ib:ib + ic].astype(np.int64),
                                                         int(prim_mat[k])))
    meshes = [np.concatenate(x) for x in per_mesh]
    car_base = len(materials)
    materials += [abi.make_material(tuple(float(x) for x in c), roughness=0.0) for c in f["car_mat_color"]]
    car = _obj_tris(f["car_pos"], f["car_nrm"], f["car_face_v"], f["car_face_n"], f["car_face_mat"] + car_base)
    light_mat = len(materials)
    materials.append(abi.make_material((100.0, 100.0, 80.0)))
    quad = quad_tris((0, -1, 0), (0, 26.0, 0), 6.9, 6.9, light_mat)
    quad.view(np.int32)[:, abi.TRI["ltriIdx"]] = [0, 1]
    car_mesh, quad_mesh = len(meshes), len(meshes) + 1
    meshes += [car, quad]
    instances = [(int(m), T) for m, T in zip(f["pica_inst_mesh"], f["pica_inst_T"])]
    light_inst = len(instances)
    instances.append((quad_mesh, np.eye(4, dtype=np.float32)))
    car_T = np.eye(4, dtype=np.float32)
    car_T[1, 3] = 5.0
    instances.append((car_mesh, car_T))
    sc = Scene(meshes=meshes, instances=instances, materials=materials, textures=textures, name="tinyapp")
    sc.area_lights = [light_from_tri(quad[i], i, light_inst, (100.0, 100.0, 80.0)) for i in range(2)]
    sc.view = camera_view((0, 0, 0), (0, 0, 1), fov_deg=40, aspect=width / height, focal=5, aperture=1e-4, distortion=0.05,
                          pixel_height=height)
    return sc
