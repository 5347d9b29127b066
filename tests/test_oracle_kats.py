"""Known-answer tests of the oracle's building blocks against independent Python/numpy restatements
of the reference formulas (tools_shared.h, platform/system.cpp, common_types.h, half.hpp)."""
import math

import numpy as np
import pytest

from lighthouse2_amd import scene
from oracle import oracle as orc


def wanghash(s):
    s &= 0xFFFFFFFF
    s = (s ^ 61) ^ (s >> 16)
    s = (s * 9) & 0xFFFFFFFF
    s = s ^ (s >> 4)
    s = (s * 0x27D4EB2D) & 0xFFFFFFFF
    return s ^ (s >> 15)


def test_wanghash_and_xorshift():
    L = orc.lib()
    rng = np.random.default_rng(0)
    for s in list(rng.integers(0, 2**32, 200)) + [0, 1, 0xFFFFFFFF, 0x12345678]:
        s = int(s)
        assert L.orc_wanghash(s) == wanghash(s)
        x = s
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        assert L.orc_xorshift(s) == x


def test_xorshift_stream_jump_ahead():
    """The vectorised generator used by the scene builder equals the sequential recurrence."""
    u = scene.xorshift_uints(0x12345678, 40000, log2b=10)
    s, ref = 0x12345678, []
    for _ in range(40000):
        s ^= (s << 13) & 0xFFFFFFFF
        s ^= s >> 17
        s ^= (s << 5) & 0xFFFFFFFF
        ref.append(s)
    assert np.array_equal(u, np.array(ref, np.uint32))


def test_bluenoise_sampler_matches_table_formula():
    """blueNoiseSampler (tools_shared.h:336-350) evaluated on the raw tables."""
    o = orc.Oracle(threads=1)
    bn = np.concatenate([o._bn.astype(np.int64), np.zeros(256, np.int64)])
    rng = np.random.default_rng(1)
    for _ in range(500):
        x, y, si, dim = (int(v) for v in rng.integers(0, [300, 300, 600, 80]))
        xx, yy, ss, dd = x & 127, y & 127, si & 255, dim & 255
        ranked = (ss ^ bn[dd + (xx + yy * 128) * 8 + 65536 * 3]) & 255
        value = bn[dd + ranked * 256] ^ bn[(dd & 7) + (xx + yy * 128) * 8 + 65536]
        ref = np.float32(np.float32(0.5) + np.float32(value)) * np.float32(1 / 256)
        assert o.L.orc_bluenoise(o.o, x, y, si, dim) == ref


def test_pack_unpack_normal_roundtrip():
    L = orc.lib()
    rng = np.random.default_rng(2)
    v = rng.normal(size=(300, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    v = v[v[:, 2] > -0.95]
    out = np.zeros(3, np.float32)
    for n in v.astype(np.float32):
        p = L.orc_pack_normal(*map(float, n))
        L.orc_unpack_normal(p, orc._fp(out))
        assert np.allclose(out, n, atol=2e-3), (n, out)


def test_mat4_inverse_matches_numpy():
    L = orc.lib()
    rng = np.random.default_rng(3)
    for _ in range(50):
        M = np.eye(4, dtype=np.float32)
        M[:3, :3] = rng.normal(size=(3, 3)).astype(np.float32) + 2 * np.eye(3, dtype=np.float32)
        M[:3, 3] = rng.normal(size=3)
        out = np.zeros(16, np.float32)
        L.orc_mat4_inverse(orc._fp(M.ravel().copy()), orc._fp(out))
        assert np.allclose(out.reshape(4, 4), np.linalg.inv(M.astype(np.float64)), rtol=1e-4, atol=1e-5)
    I = np.eye(4, dtype=np.float32).ravel().copy()
    out = np.zeros(16, np.float32)
    L.orc_mat4_inverse(orc._fp(I), orc._fp(out))
    assert np.array_equal(out, I)     # exact identity: the single-instance fast path relies on it


@pytest.mark.parametrize("fn,lo,hi,ref,tol", [
    (0, -7.0, 7.0, np.sin, 3e-7), (1, -7.0, 7.0, np.cos, 3e-7), (2, -80.0, 80.0, np.exp, 4e-7),
    (3, 1e-30, 1e30, np.log, 2e-7), (6, -1.0, 1.0, np.arccos, 4e-7)])
def test_detmath_accuracy(fn, lo, hi, ref, tol):
    rng = np.random.default_rng(fn)
    if fn == 3:
        x = np.exp(rng.uniform(np.log(lo), np.log(hi), 20000)).astype(np.float32)
    else:
        x = rng.uniform(lo, hi, 20000).astype(np.float32)
    got = orc.detmath(fn, x).astype(np.float64)
    want = ref(x.astype(np.float64))
    scale = np.maximum(np.abs(want), 1.0 if fn in (0, 1, 6) else 1e-30)
    assert np.max(np.abs(got - want) / scale) < tol * 4


def test_detmath_pow_atan2():
    rng = np.random.default_rng(7)
    x = rng.uniform(1e-6, 1.0, 20000).astype(np.float32)
    y = rng.uniform(0.0, 1.0, 20000).astype(np.float32)
    assert np.max(np.abs(orc.detmath(4, x, y) - np.power(x.astype(np.float64), y)) / np.power(x.astype(np.float64), y)) < 4e-6
    a = rng.normal(size=20000).astype(np.float32)
    b = rng.normal(size=20000).astype(np.float32)
    assert np.max(np.abs(orc.detmath(5, a, b) - np.arctan2(a.astype(np.float64), b))) < 1e-6
    # quadrant edge cases
    for (yy, xx) in [(0.0, 1.0), (1.0, 0.0), (-1.0, 0.0), (0.0, -1.0), (0.0, 0.0), (-1e-30, -1.0)]:
        v = orc.detmath(5, np.array([yy], np.float32), np.array([xx], np.float32))[0]
        assert abs(v - math.atan2(yy, xx)) < 1e-6 or (yy == 0 and xx == 0)


def test_half_conversion_matches_numpy():
    rng = np.random.default_rng(8)
    x = np.concatenate([rng.normal(scale=s, size=5000) for s in (1e-6, 1e-3, 1, 100, 3e4)]).astype(np.float32)
    x = np.concatenate([x, np.float32([0, -0.0, 65504, 65519, 65520, 1e10, 5.96e-8, 2.98e-8, 2.99e-8])])
    got = orc.detmath(7, x)
    want = x.astype(np.float16).astype(np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_saturating_float_to_uint():
    x = np.float32([-1.0, 0.0, 0.5, 1.5, 4294967040.0, 4294967296.0, 1e20, np.nan])
    got = orc.detmath(8, x)
    assert list(got) == [0.0, 0.0, 0.0, 1.0, 4294967040.0, 4294967295.0, 4294967295.0, 0.0]


def test_hit_barycentrics_follow_prime_convention():
    """Hit records carry OptiX Prime barycentrics (u = weight of vertex0, v = weight of vertex1, the
    convention material_shared.h:77-78 interpolates with): u*v0 + v*v1 + (1-u-v)*v2 = O + t*D, to the
    16-bit quantisation of the uv word (pathtracer.h:71)."""
    from lighthouse2_amd import abi
    tris = scene.random_triangles(2000, seed=7, edge=2.0)
    o = orc.Oracle(threads=2)
    o.set_materials([abi.make_material()])
    o.set_geometry(0, tris)
    o.set_instance(0, 0, None)
    o.update_toplevel()
    rng = np.random.default_rng(3)
    n = 4000
    org = (rng.normal(size=(n, 3)) * 12).astype(np.float32)
    d = (rng.uniform(-4, 4, (n, 3)) - org).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    O4 = np.concatenate([org, np.full((n, 1), 1e-4, np.float32)], 1)
    D4 = np.concatenate([d, np.full((n, 1), 1e34, np.float32)], 1)
    hits = o.trace_closest(O4, D4)
    hit = hits[:, 1] != 0xFFFFFFFF
    assert hit.mean() > 0.3
    h = hits[hit]
    u = (h[:, 3] & 0xFFFF) / 65535.0
    v = (h[:, 3] >> 16) / 65535.0
    T = tris[h[:, 1].astype(np.int64)]
    V = [T[:, abi.TRI[k]:abi.TRI[k] + 3].astype(np.float64) for k in ("vertex0", "vertex1", "vertex2")]
    P = u[:, None] * V[0] + v[:, None] * V[1] + (1 - u - v)[:, None] * V[2]
    Q = org[hit] + h[:, 0].view(np.float32)[:, None].astype(np.float64) * d[hit]
    assert np.max(np.linalg.norm(P - Q, axis=1)) < 2e-3 * 2.0


def _np_fetch(tex, u, v, o, w, h):
    """sampling_shared.h:35-64 (BILINEAR) restated in numpy float32, for one texel fetch."""
    f = np.float32
    w, h = max(w, 1), max(h, 1)
    tcx = f(f(max(f(u + f(1000)), f(0)) * f(w)) - f(0.5))
    tcy = f(f(max(f(v + f(1000)), f(0)) * f(h)) - f(0.5))
    iu, iv = int(tcx) % w, int(tcy) % h
    fu, fv = f(tcx - np.floor(tcx)), f(tcy - np.floor(tcy))
    w0, w1, w2 = f(f(1) - fu) * f(f(1) - fv), fu * f(f(1) - fv), f(f(1) - fu) * fv
    w3 = f(f(1) - f(f(w0 + w1) + w2))
    iu1, iv1 = (iu + 1) % w, (iv + 1) % h
    p = [tex[o + iu + iv * w], tex[o + iu1 + iv * w], tex[o + iu + iv1 * w], tex[o + iu1 + iv1 * w]]
    c = [np.array([(t >> s) & 255 for s in (0, 8, 16, 24)], np.float32) * f(1.0 / 256.0) for t in p]
    return ((c[0] * w0 + c[1] * w1) + c[2] * w2) + c[3] * w3


def test_fetch_texel_matches_numpy_restatement():
    """Oracle FetchTexel / FetchTexelTrilinear (sampling_shared.h:35-86) against an independent numpy
    restatement; mipmaps against a loop restatement of HostTexture::ConstructMIPmaps."""
    from lighthouse2_amd import scene
    from oracle.oracle import Oracle
    rng = np.random.default_rng(3)
    rgba = rng.integers(0, 256, (16, 32, 4), dtype=np.uint8)
    t = scene.make_texture(rgba)
    # mip level 1 by loops (host_texture.cpp:136-147)
    src = rgba.view(np.uint32).reshape(16, 32)
    lvl1 = t.pixels[32 * 16:32 * 16 + 16 * 8].reshape(8, 16)
    for y in range(8):
        for x in range(16):
            q = [int(src[2 * y, 2 * x]), int(src[2 * y, 2 * x + 1]), int(src[2 * y + 1, 2 * x]), int(src[2 * y + 1, 2 * x + 1])]
            a = min(s >> 24 for s in q)
            r, g, b = (sum((s >> k) & 255 for s in q) >> 2 for k in (16, 8, 0))
            assert lvl1[y, x] == (a << 24) + (r << 16) + (g << 8) + b
    o = Oracle()
    o.set_textures([t])
    for k in range(300):
        u, v = rng.uniform(-3, 3, 2).astype(np.float32)
        got = o.fetch_texel(0, float(u), float(v), 0, 32, 16)
        want = _np_fetch(t.pixels, np.float32(u), np.float32(v), 0, 32, 16)
        assert np.array_equal(got, want), (u, v, got, want)
    # trilinear: lambda between levels 1 and 2 = mix of the two bilinear fetches
    lam = np.float32(1.25)
    got = o.fetch_texel(0, 0.3, 0.7, 0, 32, 16, float(lam), True)
    p0 = _np_fetch(t.pixels, np.float32(0.3), np.float32(0.7), 32 * 16, 16, 8)
    p1 = _np_fetch(t.pixels, np.float32(0.3), np.float32(0.7), 32 * 16 + 16 * 8, 8, 4)
    f = np.float32(0.25)
    assert np.array_equal(got, (np.float32(1) - f) * p0 + f * p1)
