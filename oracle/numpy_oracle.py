"""oracle/numpy_oracle.py — TEST INFRASTRUCTURE ONLY.

An independent float32 restatement of res/shaders/voxel.glsl in NumPy scalars, written from the
GLSL text separately from oracle/vrt_oracle.c, used to cross-check the C oracle on small
configurations (tests/test_oracle_crosscheck.py). Each GLSL operation is one np.float32
operation (IEEE single, round to nearest), evaluated in the shader's order. It follows the same
pinned conventions as DESIGN.md "Numerics" (texture NEAREST+REPEAT as floor(c) mod N, tie index 3
clamped to 2, VRT_MAX_STEPS cap, pow = exp2(y*log2(x)), max drops NaN).

Slow (pure-Python loop per pixel): use for <= a few thousand pixels.
"""
from __future__ import annotations

import numpy as np

F = np.float32
Z = F(0.0)
ONE = F(1.0)
HALF = F(0.5)
MAX_STEPS = 4096

# voxel.glsl:71-91 (_COLOR_ONLY): refractivity, transparent, reflective, kd, ks, exp, rgba
MATERIALS = [
    (F(1.0), True, False, F(0.0), F(0.0), F(0.0), (F(0), F(0), F(0), F(0))),
    (F(1.0), False, False, F(0.4), F(0.2), F(10.0), (F(0.5), F(0.5), F(0.5), F(1.0))),
    (F(1.5), True, True, F(1.0), F(1.0), F(1.0), (F(0), F(0), F(0), F(0))),
    (F(1.0), False, False, F(0.4), F(0.2), F(10.0), (F(0.05), F(0.5), F(0.1), F(1.0))),
]
# voxel.glsl:51-68 (textured): refractivity, transparent, reflective, kd, ks, exp, (texX, texY)
MATERIALS_TEX = [
    (F(1.0), True, False, F(0.0), F(0.0), F(0.0), (0, 0)),
    (F(1.0), False, False, F(0.4), F(0.6), F(60.0), (0, 0)),
    (F(1.5), True, True, F(1.0), F(1.0), F(0.3), (0, 1)),
    (F(1.0), False, False, F(0.4), F(0.4), F(20.0), (1, 1)),
]
AMBIENT = F(0.3)
AXIS = ((0, 2, 1), (1, 0, 2), (2, 0, 1))   # intersectionAxis (:93)

M32 = 0xFFFFFFFF


def _hash(x):   # voxel.glsl:98-106
    x = (x + (x << 10)) & M32
    x ^= x >> 6
    x = (x + (x << 3)) & M32
    x ^= x >> 11
    x = (x + (x << 15)) & M32
    return x


def _bits(f):
    return int(np.array(f, dtype=np.float32).view(np.uint32))


def _random(v):   # Random(vec4) :127-130 = FloatConstruct(Hash(floatBitsToUint(v)))
    h = _hash(_bits(v[0]) ^ _hash(_bits(v[1])) ^ _hash(_bits(v[2])) ^ _hash(_bits(v[3])))
    m = (h & 0x007FFFFF) | 0x3F800000
    return np.array(m, dtype=np.uint32).view(np.float32)[()] - ONE


def v_add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def v_sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def v_scale(a, s):
    return (a[0] * s, a[1] * s, a[2] * s)


def s_scale(s, a):
    return (s * a[0], s * a[1], s * a[2])


def v_dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def v_normalize(a):
    return v_scale(a, ONE / np.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]))


def v_reflect(i, n):
    return v_sub(i, s_scale(F(2.0) * v_dot(n, i), n))


def v_refract(i, n, eta):
    d = v_dot(n, i)
    k = ONE - eta * eta * (ONE - d * d)
    if k < Z:
        return (Z, Z, Z)
    return v_sub(s_scale(eta, i), s_scale(eta * d + np.sqrt(k), n))


def g_sign(x):
    return ONE if x > Z else (F(-1.0) if x < Z else Z)


def g_min(x, y):
    return y if y < x else x


def g_max(x, y):
    if np.isnan(x):
        return y
    if np.isnan(y):
        return x
    return x if x > y else y


def g_pow(x, y):
    with np.errstate(all="ignore"):
        return np.exp2(y * np.log2(x))


def g_mix(x, y, a):
    return x * (ONE - a) + y * a


class Tracer:
    def __init__(self, vox, n, params):
        self.vox = np.asarray(vox, np.uint8)
        self.n = n
        self.size = F(n)
        self.sun = tuple(F(x) for x in params["sun_dir"])
        self.time = F(params["time"])
        self.ray_noise = F(params["ray_noise"])
        self.refl_noise = F(params["reflection_noise"])
        self.refr_noise = F(params["refraction_noise"])
        self.max_len = F(params["max_ray_length"])
        self.R = params["max_reflections"]
        self.T = params["max_transparencies"]
        self.textured = not params.get("color_only", 1)
        if self.textured:
            self.atlas = np.asarray(params["atlas"], np.uint8)   # [S, S, 4], row 0 = bottom
            self.atlas_size = int(params["atlas_size"])
            self.atlas_tex = int(params["atlas_texture_size"])
        self.mats = MATERIALS_TEX if self.textured else MATERIALS
        self.cnt = dict(pixels=0, primary_rays=0, secondary_rays=0, shadow_rays=0, dda_steps=0,
                        shadow_steps=0, refraction_probes=0, tie3=0, step_cap=0)

    def color(self, hit):
        """GetColor (:174-182): the material colour, or the atlas texel at GetTextureCoordinate
        (:167-172) of the hit's face plane (NEAREST, REPEAT, b / 255)."""
        if not self.textured:
            return MATERIALS[min(hit["voxel"], 3)][6]
        tx, ty = MATERIALS_TEX[min(hit["voxel"], 3)][6]
        ax = AXIS[hit["index"]]
        px, py = hit["point"][ax[1]], hit["point"][ax[2]]
        fx = px - F(np.floor(px))
        fy = py - F(np.floor(py))
        ts, size = F(self.atlas_tex), F(self.atlas_size)
        u = ((fx + F(tx)) * ts) / size
        v = ONE - ((((ONE - fy) + F(ty)) * ts) / size)
        S = self.atlas_size
        su, sv = u * size, v * size
        i = int(np.floor(su)) % S if su == su else 0
        j = int(np.floor(sv)) % S if sv == sv else 0
        return tuple(F(b) / F(255.0) for b in self.atlas[j, i])

    # RandomizeDirection :132-140
    def randomize(self, d, p, randomness, seed):
        q = (p[0] + d[0] + seed, p[1] + d[1] + seed, p[2] + d[2] + seed)
        r = [_random((q[0], q[1], q[2], w + seed)) for w in (Z, HALF, ONE)]
        return v_normalize(v_add(d, v_scale(v_sub(tuple(r), (HALF, HALF, HALF)), randomness)))

    # GetVoxel :149-154 -> (byte, texel index or -1)
    def get_voxel(self, c):
        s = self.size
        inside = all((x >= Z) and (x <= s) for x in c)   # NaN compares false -> outside
        if not inside:
            return 0, -1
        ijk = [int(np.floor(x)) % self.n for x in c]
        idx = ijk[0] + ijk[1] * self.n + ijk[2] * self.n * self.n
        return int(self.vox[idx]), idx

    def test_cube(self, p, d):   # :248-257, centre N/2, size N
        hi = self.size * HALF + self.size / F(2.0)
        lo = self.size * HALF - self.size / F(2.0)
        for a in range(3):
            if (p[a] > hi and d[a] > Z) or (p[a] < lo and d[a] < Z):
                return False
        return True

    @staticmethod
    def next_plane(d, p):
        return tuple(np.ceil(p[a] - ONE) if d[a] < Z else np.floor(p[a] + ONE) for a in range(3))

    def shadow_ray(self, ray, hit):   # :191-201
        return dict(pos=hit["point"], dir=v_normalize(self.sun), len=hit["len"],
                    energy=ray["energy"], voxel=hit["voxel"], r=0, t=0)

    def reflection_ray(self, ray, hit):   # :203-215
        d = self.randomize(v_reflect(ray["dir"], hit["normal"]), hit["point"], self.refl_noise,
                           self.time)
        fres = ONE - v_dot(tuple(-x for x in hit["normal"]), ray["dir"])
        return dict(pos=hit["point"], dir=d, len=hit["len"], energy=ray["energy"] * fres, voxel=0,
                    r=ray["r"] + 1, t=ray["t"])

    def refraction_ray(self, ray, hit):   # :217-246
        outv, _ = self.get_voxel(v_add(hit["point"], v_scale(hit["normal"], HALF)))
        inv, _ = self.get_voxel(v_sub(hit["point"], v_scale(hit["normal"], HALF)))
        self.cnt["refraction_probes"] += 1
        eta = self.mats[min(outv, 3)][0] / self.mats[min(inv, 3)][0]
        d = v_refract(v_normalize(ray["dir"]), hit["normal"], eta)
        if d[0] == Z and d[1] == Z and d[2] == Z:
            out = self.reflection_ray(ray, hit)
            out["voxel"] = ray["voxel"]
            out["energy"] = ray["energy"]
        else:
            e = ray["energy"]
            if ray["voxel"] == 0:
                e = e * (ONE - self.color(hit)[3])
            out = dict(pos=hit["point"], dir=self.randomize(d, hit["point"], self.refr_noise,
                                                            self.time),
                       energy=e, voxel=hit["voxel"])
        out["len"] = hit["len"]
        out["r"] = ray["r"]
        out["t"] = ray["t"] + 1
        return out

    def _step(self, ray, t, length, stats):
        """One DDA iteration (:279-286 / :323-331). Returns (t, length, cur, voxel, vidx, index)."""
        tmin = g_min(t[0], g_min(t[1], t[2]))
        t = (t[0] - tmin, t[1] - tmin, t[2] - tmin)
        length = length + tmin
        s = length - ray["len"]
        cur = v_add(ray["pos"], s_scale(s, ray["dir"]))
        eq = tuple(F(1.0) if x == Z else Z for x in t)
        step = tuple(g_sign(x) for x in ray["dir"])
        sample = v_add(cur, (HALF * eq[0] * step[0], HALF * eq[1] * step[1], HALF * eq[2] * step[2]))
        voxel, vidx = self.get_voxel(sample)
        index = int(np.floor(eq[0] * Z + eq[1] * ONE + eq[2] * F(2.0)))
        if index == 3:
            self.cnt["tie3"] += 1
            stats["flags"] |= 1
            index = 2
        return t, length, cur, voxel, vidx, index, step

    def _t_update(self, ray, t, cur, step, index, length):
        a = AXIS[index][0]
        q = ((cur[a] + step[a]) - ray["pos"][a]) / ray["dir"][a] - (length - ray["len"])
        return tuple(q if i == a else t[i] for i in range(3))

    def march_shadow(self, ray, stats):   # :259-300
        length = ray["len"]
        cur = ray["pos"]
        with np.errstate(all="ignore"):
            t = tuple((self.next_plane(ray["dir"], cur)[a] - ray["pos"][a]) / ray["dir"][a]
                      for a in range(3))
        it = 0
        while length < self.max_len:
            if not self.test_cube(cur, ray["dir"]):
                return False
            if it >= MAX_STEPS:
                self.cnt["step_cap"] += 1
                stats["flags"] |= 2
                return False
            it += 1
            stats["steps"] += 1
            self.cnt["shadow_steps"] += 1
            with np.errstate(all="ignore"):
                t, length, cur, voxel, _, index, step = self._step(ray, t, length, stats)
                if voxel != 0 and not self.mats[min(voxel, 3)][1]:
                    return True
                t = self._t_update(ray, t, cur, step, index, length)
        return False

    def march(self, ray, stats):   # :302-384; mutates `ray` (inout)
        miss = dict(found=False)
        length = ray["len"]
        cur = ray["pos"]
        with np.errstate(all="ignore"):
            t = tuple((self.next_plane(ray["dir"], cur)[a] - ray["pos"][a]) / ray["dir"][a]
                      for a in range(3))
        ray_voxel = ray["voxel"]
        internal = 0
        it = 0
        while length < self.max_len:
            if not self.test_cube(cur, ray["dir"]):
                return miss
            if it >= MAX_STEPS:
                self.cnt["step_cap"] += 1
                stats["flags"] |= 2
                return miss
            it += 1
            stats["steps"] += 1
            self.cnt["dda_steps"] += 1
            with np.errstate(all="ignore"):
                t, length, cur, voxel, vidx, index, step = self._step(ray, t, length, stats)
            a = AXIS[index][0]
            normal = [Z, Z, Z]
            normal[a] = -g_sign(ray["dir"][a])
            hit = dict(found=True, voxel=voxel, point=cur, len=length, normal=tuple(normal),
                       vidx=vidx, index=index)
            if voxel != 0 and voxel != ray_voxel:
                return hit
            if ray_voxel != 0 and voxel == 0:
                old_dir = ray["dir"]
                new = self.refraction_ray(ray, hit)
                ray.clear()
                ray.update(new)
                ray["t"] -= 1
                if ray["voxel"] == ray_voxel:
                    internal += 1
                    if internal > 10:
                        ray["dir"] = old_dir
                        ray["voxel"] = 0
                ray_voxel = ray["voxel"]
                with np.errstate(all="ignore"):
                    t = tuple((self.next_plane(ray["dir"], cur)[k] - ray["pos"][k]) / ray["dir"][k]
                              for k in range(3))
                step = tuple(g_sign(x) for x in ray["dir"])
            with np.errstate(all="ignore"):
                t = self._t_update(ray, t, cur, step, index, length)
        return miss

    def skybox(self, ray, color):   # :386-393
        u = v_normalize(ray["dir"])
        sun = F(10.0) * g_pow(v_dot(v_normalize(self.sun), u), F(400.0))
        grad = (u[1] + ONE) * HALF
        sy = g_max(self.sun[1], Z)
        sky = (g_max(Z, sun) * sy, g_max(grad * F(0.75), sun) * sy, g_max(grad, Z) * sy)
        a = ONE - ray["energy"]
        return tuple(g_mix(sky[i], color[i], a) for i in range(3))

    def trace_with_shadow(self, ray, color, stats):   # :395-423
        hit = self.march(ray, stats)
        if hit["found"]:
            sr = self.shadow_ray(ray, hit)
            self.cnt["shadow_rays"] += 1
            in_shadow = self.march_shadow(sr, stats)
            mat = self.mats[min(hit["voxel"], 3)]
            if in_shadow:
                b = AMBIENT
            else:
                diffuse = mat[3] * g_max(v_dot(hit["normal"], sr["dir"]), Z)
                spec = mat[4] * g_pow(g_max(v_dot(v_reflect(sr["dir"], hit["normal"]), ray["dir"]),
                                            Z), mat[5])
                b = AMBIENT + diffuse + spec
            rgba = self.color(hit)
            e = ray["energy"]
            color = tuple(g_mix(color[i], rgba[i] * rgba[3] * b, e) for i in range(3))
        else:
            sky = self.skybox(ray, color)
            a = ONE - ray["energy"]
            color = tuple(g_mix(sky[i], color[i], a) for i in range(3))
        return hit, color

    def pixel(self, inv_pv, w, h, px, py):   # vertex :467-472 at the pixel centre + main :425-452
        m = [F(x) for x in inv_pv]
        x = (F(2.0) * (F(px) + HALF)) / F(w) - ONE
        y = (F(2.0) * (F(py) + HALF)) / F(h) - ONE

        def mul(z):
            return [((m[0 * 4 + i] * x + m[1 * 4 + i] * y) + m[2 * 4 + i] * z) + m[3 * 4 + i] * ONE
                    for i in range(4)]

        n4, f4 = mul(F(-1.0)), mul(ONE)
        near = (n4[0] / n4[3], n4[1] / n4[3], n4[2] / n4[3])
        vdir = v_sub((f4[0] / f4[3], f4[1] / f4[3], f4[2] / f4[3]), near)
        stats = dict(steps=0, flags=0)
        color = (Z, Z, Z)
        half_n = self.size * HALF
        stack = [dict(pos=(near[0] + half_n, near[1] + half_n, near[2] + half_n),
                      dir=self.randomize(v_normalize(vdir), near, self.ray_noise, self.time),
                      len=Z, energy=ONE, voxel=0, r=0, t=0)]
        cap = self.R + self.T + 1
        self.cnt["pixels"] += 1
        self.cnt["primary_rays"] += 1
        first = True
        rec = (-1, Z)
        while stack:
            ray = stack.pop()
            if not first:
                self.cnt["secondary_rays"] += 1
            hit, color = self.trace_with_shadow(ray, color, stats)
            if first:
                if hit["found"]:
                    rec = (hit["vidx"], hit["len"])
                first = False
            if hit["found"]:
                mat = self.mats[min(hit["voxel"], 3)]
                if mat[2] and ray["r"] < self.R:
                    if len(stack) < cap:
                        stack.append(self.reflection_ray(ray, hit))
                    else:
                        stats["flags"] |= 4
                if mat[1] and ray["t"] < self.T and self.color(hit)[3] != ONE:
                    if len(stack) < cap:
                        stack.append(self.refraction_ray(ray, hit))
                    else:
                        stats["flags"] |= 4
        return color, rec, stats


def render(inv_pv, w, h, vox, n, params, rows=None):
    """Returns rgba[len(rows), w, 4], hits (structured, HIT dtype fields), counters dict."""
    tr = Tracer(vox, n, params)
    rows = list(range(h)) if rows is None else list(rows)
    rgba = np.zeros((len(rows), w, 4), np.float32)
    hits = np.zeros((len(rows), w), [("voxel_index", "<i4"), ("ray_length", "<f4"),
                                     ("steps", "<u4"), ("flags", "<u4")])
    for i, py in enumerate(rows):
        for px in range(w):
            color, rec, st = tr.pixel(inv_pv, w, h, px, py)
            rgba[i, px] = (color[0], color[1], color[2], 1.0)
            hits[i, px] = (rec[0], rec[1], st["steps"], st["flags"])
    return rgba, hits, tr.cnt


# ---- temporal filter + RGB8 store (independent restatement of oracle_temporal) ----
def unorm8(f):
    """GL float -> UNORM8 store as pinned in DESIGN.md: clamp [0,1] (NaN -> 0), *255, round half
    to even."""
    f = np.asarray(f, np.float32)
    c = np.fmin(np.fmax(f, np.float32(0.0)), np.float32(1.0))
    return np.rint(c * np.float32(255.0)).astype(np.uint8)


def temporal(rgba, prev_rgba8, alpha):
    """temporal.glsl:18 on RGB8 textures; returns (raw, cur) RGBA8 (A = 255)."""
    rgba = np.asarray(rgba, np.float32)
    prev = np.asarray(prev_rgba8, np.uint8)
    a = np.float32(alpha)
    raw = np.empty(rgba.shape, np.uint8)
    raw[..., :3] = unorm8(rgba[..., :3])
    raw[..., 3] = 255
    nw = raw[..., :3].astype(np.float32) / np.float32(255.0)
    old = prev[..., :3].astype(np.float32) / np.float32(255.0)
    cur = np.empty(rgba.shape, np.uint8)
    cur[..., :3] = unorm8(a * nw + (np.float32(1.0) - a) * old)
    cur[..., 3] = 255
    return raw, cur
