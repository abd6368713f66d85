"""Known-answer tests of the oracle's restated primitives (values derived from the formulas of
src/geometry.jl, src/shading.jl, src/math.jl, src/color.jl)."""
import ctypes as C

import numpy as np
import pytest

f32p = C.POINTER(C.c_float)


def arr(*v):
    return (C.c_float * len(v))(*v)


def tri(oracle, o, d, p1, p2, p3, tmin=1e-4, tmax=np.inf):
    out = (C.c_float * 3)()
    hit = oracle.lib.or_intersect_triangle(arr(*o), arr(*d), tmin, tmax, arr(*p1), arr(*p2), arr(*p3), out)
    return hit, tuple(out)


def test_intersect_triangle_known_answers(oracle):
    p1, p2, p3 = (0, 0, 0), (1, 0, 0), (0, 1, 0)
    hit, (u, v, t) = tri(oracle, (0.25, 0.5, 1), (0, 0, -1), p1, p2, p3)
    assert hit and (u, v, t) == (0.25, 0.5, 1.0)  # Moller-Trumbore barycentrics (geometry.jl:206)
    assert not tri(oracle, (0.75, 0.5, 1), (0, 0, -1), p1, p2, p3)[0]  # u + v > 1
    assert not tri(oracle, (0.25, 0.5, 1), (1, 0, 0), p1, p2, p3)[0]   # parallel: det == 0
    assert not tri(oracle, (0.25, 0.5, 1), (0, 0, -1), p1, p2, p3, tmax=0.5)[0]  # t > tmax
    hit, (_, _, t) = tri(oracle, (0.25, 0.5, 1), (0, 0, -1), p1, p2, p3, tmax=1.0)
    assert hit and t == 1.0  # t == tmax is accepted (reject only t > tmax)


def bbox(oracle, o, d, bmin, bmax, tmin=1e-4, tmax=np.inf):
    return oracle.lib.or_intersect_bbox(arr(*o), arr(*d), tmin, tmax, arr(*bmin), arr(*bmax))


def test_intersect_bbox_semantics(oracle):
    assert bbox(oracle, (0, 0, -5), (0, 0, 1), (-1, -1, -1), (1, 1, 1))
    assert not bbox(oracle, (3, 0, -5), (0, 0, 1), (-1, -1, -1), (1, 1, 1))
    # ray lying exactly in a slab plane with a zero direction component: 0 * Inf = NaN, and
    # Julia's NaN-propagating min/max cull the box (geometry.jl:96-105)
    assert not bbox(oracle, (1, 0, -5), (0, 0, 1), (-1, -1, -1), (1, 1, 1))
    # the Float64 tolerance t1 *= 1.00000024 accepts an entry just past the exit
    t1 = np.float32(2.0)
    t0 = np.nextafter(t1, np.float32(3))  # t0 = t1 + 1 ulp
    assert bbox(oracle, (0, 0, 0), (1, 1, 1), (float(t0), -5, -5), (float(t1) + 10, float(t1), 5))
    assert not bbox(oracle, (0, 0, 0), (1, 1, 1), (2.001, -5, -5), (12, 2.0, 5))


def fresnel(oracle, eta, n, o):
    return oracle.lib.or_fresnel_dielectric(eta, arr(*n), arr(*o))


def test_fresnel_dielectric(oracle):
    r = fresnel(oracle, 1.5, (0, 0, 1), (0, 0, 1))
    assert abs(r - ((1.5 - 1) / (1.5 + 1)) ** 2) < 1e-7  # normal incidence: 0.04
    c = np.float32(np.cos(np.radians(80)))
    assert fresnel(oracle, 1 / 1.5, (0, 0, 1), (0, float(np.sqrt(1 - c * c)), float(c))) == 1.0  # TIR


def _mix64(z):
    m = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def _pcg32_floats(seed, pixel, sample, n):
    """Independent restatement of the build's RNG: PCG32 (XSH-RR) keyed by
    SplitMix64 finalisers of (seed, pixel, sample); rand1f = (x >> 8) * 2^-24."""
    m64, mult = (1 << 64) - 1, 6364136223846793005
    key = _mix64(seed ^ _mix64((pixel << 32) | sample))
    inc = ((_mix64(key ^ 0xDA3E39CB94B95BDB) << 1) | 1) & m64
    state = ((inc + key) * mult + inc) & m64
    out = []
    for _ in range(n):
        old = state
        state = (old * mult + inc) & m64
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        x = ((xs >> rot) | (xs << ((32 - rot) & 31))) & 0xFFFFFFFF
        out.append(np.float32(x >> 8) * np.float32(2.0**-24))
    return np.array(out, np.float32)


def test_rng_stream(oracle):
    out = (C.c_float * 4096)()
    oracle.lib.or_rng_first(0x5EED, 17, 3, 4096, out)
    v = np.array(out)
    np.testing.assert_array_equal(v.astype(np.float32), _pcg32_floats(0x5EED, 17, 3, 4096))
    assert np.all((v >= 0) & (v < 1))
    assert np.all(v * 2**24 == np.floor(v * 2**24))  # 24-bit resolution like rand(Float32)
    assert abs(v.mean() - 0.5) < 0.02
    out2 = (C.c_float * 4)()
    oracle.lib.or_rng_first(0x5EED, 17, 4, 4, out2)
    assert tuple(out2) != tuple(v[:4])  # streams differ per sample


def test_inverse_frame(oracle):
    rng = np.random.default_rng(0)
    f = rng.normal(size=12).astype(np.float32)
    out = (C.c_float * 12)()
    oracle.lib.or_inverse_frame(arr(*f), 1, out)
    inv = np.array(out, np.float64)
    m = f[:9].reshape(3, 3).T.astype(np.float64)  # columns x, y, z
    mi = inv[:9].reshape(3, 3).T
    np.testing.assert_allclose(mi @ m, np.eye(3), atol=1e-5)
    np.testing.assert_allclose(mi @ f[9:] + inv[9:], 0, atol=1e-5)
    q = np.linalg.qr(rng.normal(size=(3, 3)))[0].astype(np.float32)
    g = np.concatenate([q.T.reshape(-1), [1, 2, 3]]).astype(np.float32)
    oracle.lib.or_inverse_frame(arr(*g), 0, out)  # rigid: transpose
    np.testing.assert_array_equal(np.array(out[:9], np.float32).reshape(3, 3), q.astype(np.float32))


def test_srgb_to_rgb(oracle):
    b = np.arange(256, dtype=np.uint8)
    out = (C.c_float * 256)()
    oracle.lib.or_srgb_to_rgb(b.ctypes.data_as(C.POINTER(C.c_uint8)), 256, out)
    c = b / 255.0
    ref = np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4)
    np.testing.assert_allclose(np.array(out), ref, rtol=1e-6, atol=1e-9)  # float32 evaluation
