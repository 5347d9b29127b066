"""Known-answer tests of the oracle's light sampling (CPU, no GPU) against an independent numpy float32 restatement of
CUDA/shared_kernel_code/lights_shared.h:36-261, written from the reference text operation by operation (C evaluation
order, one float32 rounding per operation, the parity contract's normalize = v * (1 / sqrtf(dot(v, v))),
include/lh2_detmath.h).  Covers every light type: the four potentials, LightPickProb with the delta lights in its sum
(the MIS weight of an implicit area-light hit, pathtracer.h:145), RandomBarycentrics, and RandomPointOnLight's pick,
point, pdf and colour for area, point, spot (a non-trivial inner / outer cone) and directional lights.

Quirks pinned here: Q2, the point light's NEE colour (lights_shared.h:228 declares a local `lightColor` that
shadows the out-parameter, so the reference leaves the caller's uninitialised float3 (pathtracer.h:183) as it was; the
restatement defines it as the light's radiance); Q3, LightPickProb of an index outside the area lights is 0; the
RenderSystem light conversions leave point / directional energy 0 (host_light.h:61, 103), so such lights are never picked.
"""
import ctypes as C

import numpy as np
import pytest

from lighthouse2_amd import scene
from oracle import oracle as orc

f32 = np.float32


def _v(a):
    return tuple(f32(x) for x in a)


def add(a, b):
    return (f32(a[0] + b[0]), f32(a[1] + b[1]), f32(a[2] + b[2]))


def sub(a, b):
    return (f32(a[0] - b[0]), f32(a[1] - b[1]), f32(a[2] - b[2]))


def smul(s, a):
    return (f32(s * a[0]), f32(s * a[1]), f32(s * a[2]))


def dot(a, b):
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def normalize(a):
    inv = f32(f32(1) / np.sqrt(dot(a, a)))
    return (f32(a[0] * inv), f32(a[1] * inv), f32(a[2] * inv))


def f3(s):
    return (f32(s.x), f32(s.y), f32(s.z))


class Lights:
    def __init__(self, area, point, spot, dirl):
        self.area, self.point, self.spot, self.dirl = area, point, spot, dirl

    # lights_shared.h:36-58
    def pot_area(self, i, O, N, I, bary):
        l = self.area[i]
        L = I
        if bary[0] >= 0:
            L = add(add(smul(bary[0], f3(l.vertex0)), smul(bary[1], f3(l.vertex1))), smul(bary[2], f3(l.vertex2)))
        L = sub(L, O)
        att = f32(f32(1) / dot(L, L))
        L = normalize(L)
        LNdotL = max(f32(0), f32(-dot(f3(l.N), L)))
        NdotL = max(f32(0), dot(N, L))
        return f32(f32(f32(f32(l.energy) * LNdotL) * NdotL) * att)

    # :64-72
    def pot_point(self, i, I, N):
        l = self.point[i]
        L = sub(f3(l.position), I)
        NdotL = max(f32(0), dot(N, L))
        att = f32(f32(1) / dot(L, L))
        return f32(f32(f32(l.energy) * NdotL) * att)

    # :78-95
    def pot_spot(self, i, I, N):
        l = self.spot[i]
        L = sub(f3(l.position), I)
        att = f32(f32(1) / dot(L, L))
        L = normalize(L)
        d = f32(f32(max(f32(0), f32(-dot(L, f3(l.direction)))) - f32(l.cosOuter)) / f32(f32(l.cosInner) - f32(l.cosOuter)))
        NdotL = max(f32(0), dot(N, L))
        LNdotL = max(f32(0), min(f32(1), d))
        e = f32(f32(f32(l.radiance.x) + f32(l.radiance.y)) + f32(l.radiance.z))
        return f32(f32(f32(e * LNdotL) * NdotL) * att)

    # :101-107
    def pot_dir(self, i, N):
        l = self.dirl[i]
        D = f3(l.direction)
        LNdotL = max(f32(0), f32(-f32(f32(f32(D[0] * N[0]) + f32(D[1] * N[1])) + f32(D[2] * N[2]))))
        return f32(f32(l.energy) * LNdotL)

    def n(self):
        return len(self.area) + len(self.point) + len(self.spot) + len(self.dirl)

    def potential(self, i, I, N, bary, areaI):
        if i < len(self.area):
            return self.pot_area(i, I, N, areaI, bary)
        i -= len(self.area)
        if i < len(self.point):
            return self.pot_point(i, I, N)
        i -= len(self.point)
        if i < len(self.spot):
            return self.pot_spot(i, I, N)
        return self.pot_dir(i - len(self.spot), N)

    # :123-138 (Q3: an index outside the area lights -> 0)
    def pick_prob(self, idx, O, N, I):
        pots = [self.potential(i, O, N, (f32(-1),) * 3, I) for i in range(self.n())]
        s = f32(0)
        for c in pots:
            s = f32(s + c)
        if s <= 0 or idx < 0 or idx >= len(self.area):
            return f32(0)
        return f32(pots[idx] / s)

    # :172-261
    def random_point(self, r0, r1, I, N):
        bary = random_barycentrics(r0)
        pots = [self.potential(i, I, N, bary, (f32(0),) * 3) for i in range(self.n())]
        s = f32(0)
        for c in pots:
            s = f32(s + c)
        if not s > 0:
            return (f32(1),) * 3, f32(0), f32(0), (f32(0),) * 3
        r1 = f32(r1 * s)
        total, idx = f32(0), 0
        for i, c in enumerate(pots):
            total = f32(total + c)
            if total >= r1:
                idx = i
                break
        pick = f32(pots[idx] / s)
        idx = min(max(idx, 0), self.n() - 1)
        na, npt, ns = len(self.area), len(self.point), len(self.spot)
        if idx < na:
            l = self.area[idx]
            P = add(add(smul(bary[0], f3(l.vertex0)), smul(bary[1], f3(l.vertex1))), smul(bary[2], f3(l.vertex2)))
            L = sub(I, P)
            sq = dot(L, L)
            L = normalize(L)
            LN = f3(l.N)
            LNdotL = f32(f32(f32(L[0] * LN[0]) + f32(L[1] * LN[1])) + f32(L[2] * LN[2]))
            reci = f32(sq / f32(f32(l.area) * LNdotL))
            pdf = reci if (LNdotL > 0 and dot(L, N) < 0) else f32(0)
            return P, pick, pdf, f3(l.radiance)
        if idx < na + npt:
            l = self.point[idx - na]
            pos = f3(l.position)
            L = sub(I, pos)
            sq = dot(L, L)
            pdf = sq if dot(L, N) < 0 else f32(0)
            return pos, pick, pdf, f3(l.radiance)          # Q2: the radiance
        if idx < na + npt + ns:
            l = self.spot[idx - na - npt]
            pos = f3(l.position)
            L = sub(I, pos)
            sq = dot(L, L)
            L = normalize(L)
            D = f3(l.direction)
            cosL = f32(f32(f32(L[0] * D[0]) + f32(L[1] * D[1])) + f32(L[2] * D[2]))
            d = f32(f32(max(f32(0), cosL) - f32(l.cosOuter)) / f32(f32(l.cosInner) - f32(l.cosOuter)))
            LNdotL = min(f32(1), d)
            pdf = f32(sq / LNdotL) if (LNdotL > 0 and dot(L, N) < 0) else f32(0)
            return pos, pick, pdf, f3(l.radiance)
        l = self.dirl[idx - na - npt - ns]
        L = f3(l.direction)
        pdf = f32(1) if dot(L, N) < 0 else f32(0)
        return sub(I, smul(f32(1000), L)), pick, pdf, f3(l.radiance)


# :145-164
def random_barycentrics(r0):
    x = f32(f32(r0) * f32(4294967296.0))
    uf = 0 if not x > 0 else min(int(x), 0xFFFFFFFF)     # Q4: saturating float -> uint
    A, B, Cc = (f32(1), f32(0)), (f32(0), f32(1)), (f32(0), f32(0))
    h = f32(0.5)

    def mid(p, q):
        return (f32(f32(p[0] + q[0]) * h), f32(f32(p[1] + q[1]) * h))
    for i in range(16):
        d = (uf >> (2 * (15 - i))) & 3
        if d == 0:
            A, B, Cc = mid(B, Cc), mid(A, Cc), mid(A, B)
        elif d == 1:
            A, B, Cc = A, mid(A, B), mid(A, Cc)
        elif d == 2:
            A, B, Cc = mid(B, A), B, mid(B, Cc)
        else:
            A, B, Cc = mid(Cc, A), mid(Cc, B), Cc
    third = f32(0.3333333)
    rx = f32(f32(f32(A[0] + B[0]) + Cc[0]) * third)
    ry = f32(f32(f32(A[1] + B[1]) + Cc[1]) * third)
    return (rx, ry, f32(f32(f32(1) - rx) - ry))


def _area_lights():
    q1 = scene.quad_tris((0, -1, 0), (-3, 6, 0), 2, 2, 1)
    q2 = scene.quad_tris((0.3, -1, 0.2), (4, 5, 1), 1.5, 3, 1)
    return [scene.light_from_tri(q[i], i, 0, rad) for q, rad in ((q1, (20, 20, 18)), (q2, (5, 9, 12))) for i in range(2)]


def _lights(kind):
    area = _area_lights()
    point = [scene.point_light((1, 4, -2), (30, 25, 20), energy=75.0), scene.point_light((-2, 3, 3), (8, 8, 8))]   # the second: RenderSystem's energy 0
    spot = [scene.spot_light((0, 7, 0), scene._norm(scene._f3(0.1, -1, 0.05)), 0.95, 0.8, (60, 50, 40)),
            scene.spot_light((-4, 4, -4), (0.5, -0.5, 0.5), 0.7, 0.69, (10, 30, 10))]   # an unnormalised direction, a thin cone edge
    dirl = [scene.directional_light(scene._norm(scene._f3(0.3, -1, 0.2)), (2, 2, 1.5), energy=5.5),
            scene.directional_light((-1, -1, -1), (255, 255, 255))]                       # apps/ai_debugger/main.cpp:63
    return {"area": (area, [], [], []), "point": ([], point, [], []), "spot": ([], [], spot, []), "dir": ([], [], [], dirl),
            "mixed": (area, point, spot, dirl), "rendersystem_delta": ([], point[1:], [], dirl[1:])}[kind]


def _oracle(lights):
    o = orc.Oracle(threads=1)
    o.set_lights(*lights)
    return o


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _samples(n, seed):
    rng = np.random.default_rng(seed)
    I = rng.uniform((-6, 0, -6), (6, 5, 6), size=(n, 3)).astype(np.float32)
    N = rng.normal(size=(n, 3))
    N /= np.linalg.norm(N, axis=1, keepdims=True)
    N[rng.random(n) < 0.5] = (0, 1, 0)          # floor-like receivers: most of them see the lights above
    return I, N.astype(np.float32), rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)


@pytest.mark.parametrize("kind", ["area", "point", "spot", "dir", "mixed", "rendersystem_delta"])
def test_random_point_on_light_matches_restatement(kind):
    lights = _lights(kind)
    ref = Lights(*lights)
    o = _oracle(lights)
    L = orc.lib()
    I, N, R0, R1 = _samples(400, hash(kind) % 1000)
    out = np.zeros(8, np.float32)
    picked = set()
    for k in range(len(I)):
        i3, n3 = np.ascontiguousarray(I[k]), np.ascontiguousarray(N[k])
        L.orc_random_point_on_light(o.o, float(R0[k]), float(R1[k]), _fp(i3), _fp(n3), _fp(out))
        P, pick, pdf, col = ref.random_point(R0[k], R1[k], _v(i3), _v(n3))
        want = np.array([*P, pick, pdf, *col], np.float32)
        assert np.array_equal(out.view(np.uint32), want.view(np.uint32)), (kind, k, out, want)
        if pdf > 0:
            picked.add(tuple(P))
    if kind == "rendersystem_delta":
        # energy 0 on both delta lights (RenderSystem's conversion): nothing is ever picked, no shadow ray is queued
        assert not picked
    else:
        assert len(picked) >= 2 or kind in ("point", "dir")


@pytest.mark.parametrize("kind", ["area", "mixed"])
def test_light_pick_prob_matches_restatement(kind):
    """LightPickProb (the MIS weight of a path that hits an area light after a non-specular bounce): the sum runs over the
    potentials of every light type; an index outside the area lights gives 0 (Q3)."""
    lights = _lights(kind)
    ref = Lights(*lights)
    o = _oracle(lights)
    L = orc.lib()
    I, N, _, _ = _samples(300, 11)
    rng = np.random.default_rng(12)
    nonzero = 0
    for k in range(len(I)):
        idx = int(rng.integers(-1, ref.n() + 1))
        li = ref.area[max(0, min(idx, len(ref.area) - 1))]
        w = rng.random(3).astype(np.float32)
        w /= w.sum()
        hit = (w[0] * np.float32([li.vertex0.x, li.vertex0.y, li.vertex0.z]) + w[1] * np.float32([li.vertex1.x, li.vertex1.y, li.vertex1.z])
               + w[2] * np.float32([li.vertex2.x, li.vertex2.y, li.vertex2.z])).astype(np.float32)
        o3, n3 = np.ascontiguousarray(I[k]), np.ascontiguousarray(N[k])
        got = L.orc_light_pick_prob(o.o, idx, _fp(o3), _fp(n3), _fp(hit))
        want = ref.pick_prob(idx, _v(o3), _v(n3), _v(hit))
        assert np.float32(got).view(np.uint32) == want.view(np.uint32), (k, idx, got, want)
        nonzero += want > 0
    assert nonzero > 50


def test_light_potentials_every_type():
    lights = _lights("mixed")
    ref = Lights(*lights)
    o = _oracle(lights)
    L = orc.lib()
    I, N, R0, _ = _samples(100, 21)
    for k in range(len(I)):
        bary = np.float32(random_barycentrics(R0[k]))
        i3, n3 = np.ascontiguousarray(I[k]), np.ascontiguousarray(N[k])
        zero = np.zeros(3, np.float32)
        for i in range(ref.n()):
            got = L.orc_light_potential(o.o, i, _fp(i3), _fp(n3), _fp(bary), _fp(zero))
            want = ref.potential(i, _v(i3), _v(n3), _v(bary), _v(zero))
            assert np.float32(got).view(np.uint32) == want.view(np.uint32), (k, i, got, want)


def test_random_barycentrics():
    L = orc.lib()
    out = np.zeros(3, np.float32)
    rng = np.random.default_rng(5)
    for r0 in list(rng.random(500).astype(np.float32)) + [np.float32(0), np.float32(0.99999994), np.float32(0.25)]:
        L.orc_random_barycentrics(float(r0), _fp(out))
        want = np.float32(random_barycentrics(r0))
        assert np.array_equal(out.view(np.uint32), want.view(np.uint32)), (r0, out, want)
        assert np.all(out >= -1e-6) and abs(out.sum() - 1) < 1e-5


def test_point_light_colour_is_its_radiance():
    """Q2 (lights_shared.h:228): with only a point light, every NEE sample that connects carries the light's radiance as
    its colour (the restatement's definition of the reference's shadowed out-parameter)."""
    p = scene.point_light((0, 5, 0), (3, 5, 7), energy=15.0)
    o = _oracle(([], [p], [], []))
    L = orc.lib()
    out = np.zeros(8, np.float32)
    i3, n3 = np.float32([0.5, 0, 0.2]), np.float32([0, 1, 0])
    L.orc_random_point_on_light(o.o, 0.3, 0.7, _fp(i3), _fp(n3), _fp(out))
    assert out[4] > 0 and tuple(out[5:8]) == (3, 5, 7) and tuple(out[:3]) == (0, 5, 0) and out[3] == 1
