"""Known-answer tests pinning the CPU oracle (oracle/vrt_oracle.c) to res/shaders/voxel.glsl.

The reference ships no tests or golden vectors, so every expected value here is
derived by hand from the GLSL formula it cites.
"""
import struct

import numpy as np
import pytest

import oracle


def f2u(f):
    return struct.unpack("<I", struct.pack("<f", f))[0]


# --- hash RNG, voxel.glsl:98-140 -----------------------------------------------------------------

@pytest.mark.parametrize("x,h", [(0, 0x00000000), (1, 0x124EA49D), (2, 0x249DC93B),
                                 (0xDEADBEEF, 0x6C7328FE)])
def test_hash1_kat(built, x, h):
    assert oracle.hash1(x) == h


def test_hash4_and_float_construct_kat(built):
    h = oracle.hash4(f2u(1.0), f2u(2.0), f2u(3.0), f2u(0.0))
    assert h == 0x772B9AE1
    assert np.float32(oracle.float_construct(h)) == np.float32(0.34066403)
    assert oracle.float_construct(0) == 0.0
    assert np.float32(oracle.float_construct(0xFFFFFFFF)) == np.float32(1.0) - np.float32(2 ** -23)


def test_randomize_direction_zero_noise_keeps_direction(built):
    # normalize(dir + (r - 0.5) * 0): a unit direction with no zero component survives bit-exact
    # up to the re-normalisation (voxel.glsl:139).
    d = np.array([0.6, -0.8, 0.0], np.float32)
    out = oracle.randomize_direction(d, [1.0, 2.0, 3.0], 0.0, 1.0)
    inv = np.float32(1) / np.sqrt(np.float32(d[0] * d[0] + d[1] * d[1]) + np.float32(0) * np.float32(0))
    np.testing.assert_array_equal(out[:2], (d * inv)[:2])
    assert out[2] == 0.0


def test_randomize_direction_noise_is_bounded(built):
    d = np.array([0.0, 0.0, 1.0], np.float32)
    out = oracle.randomize_direction(d, [5.0, 6.0, 7.0], 0.05, 3.0)
    assert abs(np.linalg.norm(out) - 1) < 1e-6
    assert np.all(np.abs(out[:2]) <= 0.026)


# --- refract / TIR (GLSL 4.50 refract, voxel.glsl:226-229) ---------------------------------------

def glsl_refract(i, n, eta):
    i = np.asarray(i, np.float32)
    n = np.asarray(n, np.float32)
    eta = np.float32(eta)
    d = np.float32(np.float32(n[0] * i[0] + n[1] * i[1]) + n[2] * i[2])
    k = np.float32(1) - eta * eta * (np.float32(1) - d * d)
    if k < 0:
        return np.zeros(3, np.float32)
    s = eta * d + np.sqrt(k)
    return eta * i - s * n


def test_refract_matches_spec_formula(built):
    i = np.array([0.6, -0.8, 0.0], np.float32)
    n = np.array([0.0, 1.0, 0.0], np.float32)
    np.testing.assert_array_equal(oracle.refract(i, n, 1 / 1.5), glsl_refract(i, n, 1 / 1.5))


def test_refract_total_internal_reflection_is_zero(built):
    i = np.array([0.8, -0.6, 0.0], np.float32)   # 53 deg from the normal, glass -> air
    n = np.array([0.0, 1.0, 0.0], np.float32)
    out = oracle.refract(i, n, 1.5)
    assert np.all(out == 0.0)


# --- DDA on hand-built volumes (RayMarch, voxel.glsl:302-384) -------------------------------------

def vol4():
    return np.zeros(4 * 4 * 4, np.uint8)


def idx(x, y, z, n=4):
    return x + y * n + z * n * n


def test_dda_axis_aligned_hit(built):
    v = vol4()
    v[idx(2, 1, 1)] = 1
    r = oracle.march_one(v, 4, [0.5, 1.5, 1.5], [1.0, 0.0, 0.0])
    # t.x: 0.5 then 1.0 -> hit the x=2 face at length 1.5 after 2 steps
    assert r["found"] and r["vidx"] == idx(2, 1, 1)
    assert r["len"] == 1.5 and r["steps"] == 2
    np.testing.assert_array_equal(r["point"], [2.0, 1.5, 1.5])
    np.testing.assert_array_equal(r["normal"], [-1.0, 0.0, 0.0])


def test_dda_negative_direction(built):
    v = vol4()
    v[idx(0, 2, 3)] = 3
    r = oracle.march_one(v, 4, [3.25, 2.5, 3.5], [-1.0, 0.0, 0.0])
    assert r["found"] and r["vidx"] == idx(0, 2, 3)
    assert r["len"] == 2.25
    np.testing.assert_array_equal(r["normal"], [1.0, 0.0, 0.0])


def test_dda_glass_is_a_hit_from_air(built):
    v = vol4()
    v[idx(1, 1, 2)] = 2
    r = oracle.march_one(v, 4, [1.5, 1.5, 0.25], [0.0, 0.0, 1.0])
    assert r["found"] and r["vidx"] == idx(1, 1, 2) and r["len"] == 1.75


def test_dda_xy_tie_steps_diagonally(built):
    # normalize((1,1,0)) has equal x and y: t.x == t.y every step -> index = 1 (y) and the sample
    # is offset on both axes (voxel.glsl:328-331), so the ray enters the diagonal neighbour.
    v = vol4()
    v[idx(1, 1, 0)] = 1
    d = np.array([1.0, 1.0, 0.0], np.float32)
    d = d * (np.float32(1) / np.sqrt(np.float32(2)))
    r = oracle.march_one(v, 4, [0.5, 0.5, 0.5], d)
    assert r["found"] and r["vidx"] == idx(1, 1, 0)
    np.testing.assert_array_equal(r["normal"], [0.0, -1.0, 0.0])


def test_dda_repeat_wrap_at_n(built):
    # A ray skimming y == N exactly is inside the `>` bounds test and reads texel row 0 (GL_REPEAT).
    v = vol4()
    v[idx(2, 0, 1)] = 1
    r = oracle.march_one(v, 4, [0.5, 4.0, 1.5], [1.0, 0.0, 0.0])
    assert r["found"] and r["vidx"] == idx(2, 0, 1) and r["len"] == 1.5


def test_dda_leaves_cube(built):
    v = vol4()
    r = oracle.march_one(v, 4, [0.5, 1.5, 1.5], [1.0, 0.0, 0.0])
    # planes 1,2,3,4 and 5: at x == 4 TestCube's strict `>` (voxel.glsl:251) keeps the ray in
    assert not r["found"] and r["steps"] == 5


def test_dda_enters_from_outside(built):
    v = vol4()
    v[idx(0, 1, 1)] = 1
    r = oracle.march_one(v, 4, [-2.5, 1.5, 1.5], [1.0, 0.0, 0.0])
    assert r["found"] and r["vidx"] == idx(0, 1, 1) and r["len"] == 2.5


def test_dda_max_ray_length(built):
    v = vol4()
    v[idx(3, 1, 1)] = 1
    # `while (rayLength < u_MaxRayLength)` tests BEFORE the step (voxel.glsl:317): at 1.5 the walk
    # stops before reaching x=3; at 2.0 it still takes the step that lands on x=3 (length 2.5).
    r = oracle.march_one(v, 4, [0.5, 1.5, 1.5], [1.0, 0.0, 0.0], max_len=1.5)
    assert not r["found"]
    r = oracle.march_one(v, 4, [0.5, 1.5, 1.5], [1.0, 0.0, 0.0], max_len=2.0)
    assert r["found"] and r["len"] == 2.5


# --- scene producers (main.cpp:218-288) ------------------------------------------------------------

def test_glass_cube_scene(built):
    n = 16
    v = oracle.build_scene(1, n).reshape(n, n, n)  # [z][y][x]
    assert v[0, 5, 5] == 2 and v[n - 1, 5, 5] == 2 and v[5, 0, 5] == 2 and v[5, n - 1, 5] == 2
    assert v[5, 5, 0] == 2 and v[5, 5, n - 1] == 2
    assert v[n // 2, n // 2, n // 2] == 3
    assert (v[1:-1, 1:-1, 1:-1] != 0).sum() == 1


def test_refraction_scene(built):
    n = 16
    v = oracle.build_scene(2, n).reshape(n, n, n)
    assert v[n // 2, n // 2, n // 2] == 2
    assert v[n // 4, n // 4, 0] == 3 and v[3 * n // 4 - 1, 3 * n // 4 - 1, 0] == 3
    assert v[n // 4 - 1, n // 4, 0] == 0
    assert np.bincount(v.reshape(-1), minlength=4)[3] == 6 * (n // 2) ** 2


def test_terrain_scene_structure(built):
    for n in (16, 64, 128):
        v = oracle.build_scene(0, n).reshape(n, n, n)
        noise = oracle.terrain_noise(n).reshape(n, n)   # [z][x]
        z, x = 3, 5
        h = np.float32(noise[z, x]) * np.float32(n)
        g = int(h)
        assert v[z, g, x] == 3
        assert all(v[z, y, x] == 1 for y in range(g))
        has_glass = (v == 2).any()
        assert has_glass == (n <= 64)   # glass walls only when size <= 64 (main.cpp:233)
