// vrt_render.hip — gfx950 HIP kernels for the per-pixel program of res/shaders/voxel.glsl; the
// C-ABI context around them is vrt_context.cpp (include/vrt.h).
//
// One work-item per pixel; a 128-thread workgroup covers a 16x8 pixel tile and each wave64 an
// 8x8 sub-tile, so the 64 rays of a wave start coherent. Every float operation of the DDA is
// replayed in the reference's order with -ffp-contract=off and correctly rounded div/sqrt, which
// makes hit records bit-exact against the CPU oracle (DESIGN.md "Numerics").
//
// Device volume layout: (N+1)^3 bytes, x fastest, where plane N repeats plane 0 on each axis.
// GetVoxel's texel for a coordinate c in [0, N] is then simply floor(c) (GL_REPEAT folded into
// the layout), and the hot loop addresses it with two 24-bit multiply-adds.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "vrt.h"
#include "vrt_internal.h"

// Diagnostic instrumentation (per-wave timestamps, certified-walk outcome counts; images and
// counters unchanged) exists only in `make variant` builds, never in the product library.
#if (defined(VRT_STAMPS) || defined(VRT_CERT_DIAG) || defined(VRT_CERT_TRACE)) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_STAMPS / VRT_CERT_DIAG are diagnostic builds: use make variant"
#endif

// VRT_DIAG_PHASE (diagnostic builds only; wrong images): the certified pass stops after phase
// 0 ray setup skipped / 1 primary ray / 2 primary certified walk / 3 shading without the shadow
// walk, for a per-phase instruction budget by PMC differences (scripts/phase_budget.py)
#if defined(VRT_DIAG_PHASE) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_DIAG_PHASE is a diagnostic build: use make variant"
#endif
#ifndef VRT_DIAG_PHASE
#define VRT_DIAG_PHASE 9
#endif
// VRT_TREE_CUT (diagnostic builds only; images stay exact): certified trees give up (exact path)
// at bit 0 reflection children, bit 1 refraction children, bit 2 in-volume refraction restarts
#if defined(VRT_TREE_CUT) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_TREE_CUT is a diagnostic build: use make variant"
#endif
#ifndef VRT_TREE_CUT
#define VRT_TREE_CUT 0
#endif
// VRT_PREFIX (A/B builds only): 0 turns off the certified prefix of the exact primary walk
#if defined(VRT_PREFIX) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_PREFIX is an A/B knob of make variant builds"
#endif
#ifndef VRT_PREFIX
#define VRT_PREFIX 1
#endif

namespace vrt {

// ------------------------------------------------------------------ GLSL vector semantics --

struct f3 {
  float x, y, z;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float comp(f3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
__device__ __forceinline__ void set_comp(f3& a, int i, float f) {
  if (i == 0) a.x = f;
  else if (i == 1) a.y = f;
  else a.z = f;
}
// RN(1 / d) from the hardware reciprocal (within 1 ulp) and one Newton step on its exact residual
// (e = 1 - d y by fma): bit-identical to the IEEE division 1.0f / d for every d with a biased
// exponent in [2, 252], i.e. |d| in [2^-125, 2^126) (exhaustive over all 2^32 bit patterns on the
// GPU, 4 211 080 714 of them in that range, 0 mismatches: vrt_debug_fast_math,
// tests/test_gpu_fast_math.py); 3 VALU instead of the division's 11. Operands the caller cannot
// bound take rcp_rn (exponent test, else the division).
__device__ __forceinline__ bool rcp_rn_ok(float d) {
  const uint32_t e = (__float_as_uint(d) >> 23) & 0xFFu;
  return e >= 2u && e <= 252u;
}
__device__ __forceinline__ float rcp_newton(float d) {
  const float y = __builtin_amdgcn_rcpf(d);
  return __builtin_fmaf(__builtin_fmaf(-d, y, 1.0f), y, y);
}
__device__ __forceinline__ float rcp_rn(float d) { return rcp_rn_ok(d) ? rcp_newton(d) : 1.0f / d; }
// RN(sqrt(s)) for s with a biased exponent in [95, 252], i.e. s in [2^-32, 2^126): the hardware
// square root moved to the neighbour its fma residuals pick (the correctly rounded sequence without
// the scaling of s < 2^-32 and the special-value select, which such s never need): bit-identical
// to the IEEE square root on every such s (exhaustive, vrt_debug_fast_math; below 2^-32 the
// unscaled hardware root is off by more than the fix can mend: 2.2 M mismatches when [2^-125,
// 2^-32) was included). Other s take the IEEE square root.
__device__ __forceinline__ bool sqrt_fix_ok(float s) {
  const uint32_t e = (__float_as_uint(s) >> 23) & 0xFFu;
  return e >= 95u && e <= 252u;
}
__device__ __forceinline__ float sqrt_fix(float s) {
  const float y = __builtin_amdgcn_sqrtf(s);
  const float ym = __uint_as_float(__float_as_uint(y) - 1u), yp = __uint_as_float(__float_as_uint(y) + 1u);
  const float rm = __builtin_fmaf(-ym, y, s), rp = __builtin_fmaf(-yp, y, s);
  const float z = rm <= 0.0f ? ym : y;
  return rp > 0.0f ? yp : z;
}
__device__ __forceinline__ float sqrt_rn(float s) { return sqrt_fix_ok(s) ? sqrt_fix(s) : __builtin_sqrtf(s); }

// RN(1 / RN(sqrt(s))) for s within 1024 ulps of 1 (bits b), in closed form: for s = 1 + k 2^-23
// (k >= 0) the correctly rounded square root is 1 + floor(k/2) 2^-23 and its reciprocal
// 1 - floor(k/2) 2^-23; for s = 1 - k 2^-24 they are 1 - ceil(k/2) 2^-24 and 1 + ceil(m/2) 2^-23,
// m = ceil(k/2) (the square root and the reciprocal sit within m^2 2^-48 of those grid points or
// midpoints, on the side that decides the rounding). Exact for |k| < 2898 (exhaustive against
// IEEE sqrt and division: tests/test_normalize_fast.py); a normalised vector's squared length is
// within a few ulps of 1, so RandomizeDirection's, the skybox's and GetRefractionRay's
// normalize of an already normalised direction takes ~6 VALU instead of ~26.
__device__ __forceinline__ float near_one_rsqrt(uint32_t b) {
  const uint32_t one = 0x3F800000u;
  const uint32_t r = b >= one ? (b - one < 2u ? one : one - ((b - one) & ~1u))
                              : one + (((((one - b) + 1u) >> 1) + 1u) >> 1);
  return __uint_as_float(r);
}
__device__ __forceinline__ f3 normalize3(f3 v) {
  const float s = v.x * v.x + v.y * v.y + v.z * v.z;
  const uint32_t b = __float_as_uint(s);
  const float inv = b - (0x3F800000u - 1024u) <= 2048u ? near_one_rsqrt(b) : rcp_rn(sqrt_rn(s));
  return v * inv;
}
__device__ __forceinline__ float gsign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
__device__ __forceinline__ float gmin(float x, float y) { return y < x ? y : x; }
__device__ __forceinline__ float gmax(float x, float y) { return __builtin_fmaxf(x, y); }
__device__ __forceinline__ float gpow(float x, float y) { return exp2f(y * log2f(x)); }
__device__ __forceinline__ float mixf(float x, float y, float a) { return x * (1.0f - a) + y * a; }
__device__ __forceinline__ f3 reflect3(f3 i, f3 n) {
  const float s = 2.0f * dot3(n, i);
  return i - s * n;
}
__device__ __forceinline__ f3 refract3(f3 i, f3 n, float eta) {
  const float d = dot3(n, i);
  const float k = 1.0f - eta * eta * (1.0f - d * d);
  if (k < 0.0f) return mk(0.0f, 0.0f, 0.0f);
  const float s = eta * d + sqrt_rn(k);
  return eta * i - s * n;
}
__device__ __forceinline__ f3 sign3(f3 d) { return mk(gsign(d.x), gsign(d.y), gsign(d.z)); }

// Jenkins one-at-a-time mix, voxel.glsl:98-125
__device__ __forceinline__ uint32_t hash1(uint32_t x) {
  x += (x << 10u);
  x ^= (x >> 6u);
  x += (x << 3u);
  x ^= (x >> 11u);
  x += (x << 15u);
  return x;
}
__device__ __forceinline__ float random4(float x, float y, float z, float w) {
  const uint32_t h = hash1(__float_as_uint(x) ^ hash1(__float_as_uint(y)) ^
                           hash1(__float_as_uint(z)) ^ hash1(__float_as_uint(w)));
  return __uint_as_float((h & 0x007FFFFFu) | 0x3F800000u) - 1.0f;
}
// RandomizeDirection, voxel.glsl:132-140 (runs even at noise 0: it decides the sign of zeros)
// With randomness == ±0 (every bench config) the added vector is (±0, ±0, ±0), and dir + r equals
// dir bit for bit (x + ±0 = x for x != 0, +0 + ±0 = +0) unless a component is -0.0 (-0 + +0 = +0)
// or NaN: only then do the hashes decide the result, so only then are they computed. Exact.
__device__ __forceinline__ bool zero_noise_exact(f3 d) {
  const uint32_t nz = 0x80000000u;
  return int(__float_as_uint(d.x) != nz) & int(__float_as_uint(d.y) != nz) &
         int(__float_as_uint(d.z) != nz) & int(d.x == d.x) & int(d.y == d.y) & int(d.z == d.z);
}
__device__ __forceinline__ f3 randomize(f3 dir, f3 pos, float randomness, float seed) {
  f3 r = mk(0.0f, 0.0f, 0.0f);
  if (!(randomness == 0.0f && zero_noise_exact(dir))) {
    const f3 p = mk((pos.x + dir.x) + seed, (pos.y + dir.y) + seed, (pos.z + dir.z) + seed);
    const float dx = random4(p.x, p.y, p.z, 0.0f + seed);
    const float dy = random4(p.x, p.y, p.z, 0.5f + seed);
    const float dz = random4(p.x, p.y, p.z, 1.0f + seed);
    r = mk((dx + -0.5f) * randomness, (dy + -0.5f) * randomness, (dz + -0.5f) * randomness);
  }
  return normalize3(dir + r);
}

// ------------------------------------------------------- materials (_COLOR_ONLY, :71-91) ----

__device__ __forceinline__ uint32_t mat_id(uint32_t b) { return b > 3 ? 3 : b; }
__device__ __forceinline__ float mat_refr(uint32_t b) { return mat_id(b) == 2 ? 1.5f : 1.0f; }
__device__ __forceinline__ bool mat_transparent(uint32_t m) { return m == 0 || m == 2; }
__device__ __forceinline__ bool mat_reflective(uint32_t m) { return m == 2; }
__device__ __forceinline__ float mat_kd(uint32_t m) { return m == 0 ? 0.0f : (m == 2 ? 1.0f : 0.4f); }
// specular factor / exponent: _COLOR_ONLY table (:83-86) or the textured table (:64-67)
__device__ __forceinline__ float mat_ks(uint32_t m, bool tex) {
  return m == 0 ? 0.0f : (m == 2 ? 1.0f : (tex ? (m == 1 ? 0.6f : 0.4f) : 0.2f));
}
__device__ __forceinline__ float mat_exp(uint32_t m, bool tex) {
  return m == 0 ? 0.0f : (m == 2 ? (tex ? 0.3f : 1.0f) : (tex ? (m == 1 ? 60.0f : 20.0f) : 10.0f));
}
// atlas slot (texX, texY) of the textured table (:64-67)
__device__ __forceinline__ uint32_t mat_tex_x(uint32_t m) { return m == 3 ? 1u : 0u; }
__device__ __forceinline__ uint32_t mat_tex_y(uint32_t m) { return m >= 2 ? 1u : 0u; }
__device__ __forceinline__ float4 mat_color(uint32_t m) {
  if (m == 1) return make_float4(0.5f, 0.5f, 0.5f, 1.0f);
  if (m == 3) return make_float4(0.05f, 0.5f, 0.1f, 1.0f);
  return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

constexpr float kAmbient = 0.3f;

// Colour-only glass (voxel.glsl:85: colour vec4(0)) adds col.rgb * col.a * brightness = +0 for any
// finite brightness (glass's lit brightness is finite: kd = ks = 1, exponent 1; RayColor, :184-188),
// so a glass hit's colour does not depend on its shadow bit: the stats-free paths skip its shadow
// walk (TraceWithShadow, :400-402). Images unchanged.
__device__ __forceinline__ bool shadow_free_hit(uint32_t byte, bool tex) { return !tex && mat_id(byte) == 2u; }

// ----------------------------------------------------------------------------- ray state --

struct Ray {
  f3 pos, dir;
  float len, energy;
  uint32_t voxel;  // byte value of the medium the ray travels in (0 = air)
  int32_t rdepth, tdepth;
};

struct Hit {
  f3 point, normal;
  float len;
  uint32_t voxel;
  int32_t vidx;  // canonical index x + y*N + z*N*N of the texel read
  int32_t axis;  // intersectionAxis row of the step (tie 3 clamped to 2)
  bool found;
};

struct Counters {
  uint32_t c[VRT_CNT_COUNT];
};

// Crossed-axis operands of a skip step come from a per-lane LDS table (one ds_read_b128 at an
// address selected from the lane's three entry addresses: 2 VALU) instead of three 3-way register
// selects. Lane-major layout: entry a of work-item t at [3t + a] (an axis-major table measured
// neutral, profiles/r01_v37_ab_axis_major_len0_cmpt.log).
constexpr int kAxStride = 1;  // float4s between axes
constexpr int kAxLane = 3;    // float4s between lanes

struct Ctx {
  const uint16_t* __restrict__ vox;  // padded (N+1)^3 layout, voxel | G << 8, one per octant (see pack kernels)
  uint32_t ostride;  // bytes between the octant volumes (0: a single centred-distance volume)
  int32_t n;
  uint32_t p;  // N + 1
  float fn;
  float max_len;
  f3 sun_n, sun_rcp;
  float sky_sy;
  float time, refl_noise, refr_noise;
  float4* ax;  // this lane's 3-entry axis table in LDS: {pos, dir, rcp, sign} per axis
  const uint32_t* atlas;  // textured instances only (TEX)
  uint32_t atlas_mask;   // atlas_size - 1 (power of two)
  float atlas_fs, atlas_fts;  // (float)u_AtlasSize, (float)u_AtlasTextureSize
#ifdef VRT_CERT_TRACE
  bool tr;  // diagnostic build: this lane's pixel is the traced one
#endif
};
#ifdef VRT_CERT_TRACE  // diagnostic build: one pixel's certified walks, 8 floats per record
__device__ float g_ctrace[1024][8];
__device__ unsigned int g_ctrace_n;
#define CTRACE(c, a0, a1, a2, a3, a4, a5, a6, a7)                                                   \
  do {                                                                                              \
    if ((c).tr) {                                                                                   \
      const unsigned int q_ = atomicAdd(&g_ctrace_n, 1u);                                           \
      if (q_ < 1024u) {                                                                             \
        g_ctrace[q_][0] = float(a0); g_ctrace[q_][1] = float(a1); g_ctrace[q_][2] = float(a2);       \
        g_ctrace[q_][3] = float(a3); g_ctrace[q_][4] = float(a4); g_ctrace[q_][5] = float(a5);       \
        g_ctrace[q_][6] = float(a6); g_ctrace[q_][7] = float(a7);                                    \
      }                                                                                             \
    }                                                                                               \
  } while (0)
#else
#define CTRACE(c, a0, a1, a2, a3, a4, a5, a6, a7) ((void)0)
#endif

// a*b + c on the low 24 bits of a and b: one v_mad_u32_u24 (operands < 2^24 for N <= 1024).
// b is wave-uniform (the padded pitch) and goes in as the instruction's one SGPR operand.
__device__ __forceinline__ uint32_t mad24(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
  return r;
}

// 16-bit load at a 32-bit byte offset from a wave-uniform base: global_load_ushort with an SGPR
// base (no 64-bit address arithmetic per lane)
__device__ __forceinline__ uint32_t load_u16(const uint16_t* __restrict__ base, uint32_t idx) {
  return *reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(base) + (idx << 1));
}
// the same texel in the volume of the ray's direction octant, `obase` bytes after the first one:
// the byte offset (idx << 1) + obase is one v_lshl_add_u32, as the plain shift was
__device__ __forceinline__ uint32_t load_u16_at(const uint16_t* __restrict__ base, uint32_t idx,
                                                uint32_t obase) {
  return *reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(base) + ((idx << 1) + obase));
}
// texel fields of the packed word: voxel byte and the skip distance (forward distance G of the
// octant, or the centred Chebyshev D of the single-volume layout; see the skip walk)
constexpr uint32_t kVoxMask = 0xFFu;
constexpr uint32_t kDistShift = 8u;

__device__ __forceinline__ int32_t canonical_index(const Ctx& c, uint32_t i, uint32_t j, uint32_t k) {
  const uint32_t n = uint32_t(c.n);
  i = i == n ? 0u : i;
  j = j == n ? 0u : j;
  k = k == n ? 0u : k;
  return int32_t(i + (j + k * n) * n);
}

// GetVoxel (voxel.glsl:149-154): `>` bounds test, NEAREST + GL_REPEAT, NaN reads 0. Reference
// form, used off the hot loop (refraction probes).
__device__ __forceinline__ uint32_t get_voxel(const Ctx& c, f3 p) {
  if (!(p.x >= 0.0f && p.y >= 0.0f && p.z >= 0.0f && p.x <= c.fn && p.y <= c.fn && p.z <= c.fn))
    return 0u;
  const uint32_t i = uint32_t(__builtin_floorf(p.x));
  const uint32_t j = uint32_t(__builtin_floorf(p.y));
  const uint32_t k = uint32_t(__builtin_floorf(p.z));
  return load_u16(c.vox, mad24(mad24(k, c.p, j), c.p, i)) & kVoxMask;
}

// TestCube (voxel.glsl:248-257) with centre N/2 and size N; bitwise ops, no short-circuit branches.
__device__ __forceinline__ bool test_cube(f3 p, f3 d, float fn) {
  const float hi = fn * 0.5f + fn / 2.0f, lo = fn * 0.5f - fn / 2.0f;
  const bool out = (p.x > hi & d.x > 0.0f) | (p.x < lo & d.x < 0.0f) | (p.y > hi & d.y > 0.0f) |
                   (p.y < lo & d.y < 0.0f) | (p.z > hi & d.z > 0.0f) | (p.z < lo & d.z < 0.0f);
  return !out;
}

__device__ __forceinline__ float next_plane(float d, float p) {
  return d < 0.0f ? __builtin_ceilf(p - 1.0f) : __builtin_floorf(p + 1.0f);
}

__device__ __forceinline__ f3 initial_t(f3 dir, f3 cur, f3 pos) {
  return mk((next_plane(dir.x, cur.x) - pos.x) / dir.x, (next_plane(dir.y, cur.y) - pos.y) / dir.y,
            (next_plane(dir.z, cur.z) - pos.z) / dir.z);
}

__device__ __forceinline__ float sel3(int axis, float x, float y, float z) {
  return axis == 2 ? z : (axis == 1 ? y : x);
}

// a / d correctly rounded, given y = RN(1/d) (Markstein's theorem: q1 is within one ulp of a/d,
// so r1 = a - d*q1 is exact and RN(q1 + r1*y) = RN(a/d); no over/underflow for the fast-path
// operand ranges, see fast_path_ok). Bit-identical to IEEE division, 5 VALU ops instead of the
// ~11 of the scaled div_scale/div_fmas/div_fixup sequence.
__device__ __forceinline__ float div_rn(float a, float d, float y) {
  const float q0 = a * y;
  const float r0 = __builtin_fmaf(-d, q0, a);
  const float q1 = __builtin_fmaf(r0, y, q0);
  const float r1 = __builtin_fmaf(-d, q1, a);
  return __builtin_fmaf(r1, y, q1);
}

// The fast walk needs every direction component normal and not tiny: then every t stays finite
// and never -0 (so v_min3 == GLSL min) and div_rn is exact. Otherwise (a +-0 component: +-inf /
// NaN t values, where the GLSL would spin) the walk replays the reference literally.
__device__ __forceinline__ bool fast_path_ok(f3 d) {
  const float lo = 0x1p-64f;
  return __builtin_fabsf(d.x) >= lo && __builtin_fabsf(d.y) >= lo && __builtin_fabsf(d.z) >= lo &&
         __builtin_fabsf(d.x) <= 1.0e4f && __builtin_fabsf(d.y) <= 1.0e4f &&
         __builtin_fabsf(d.z) <= 1.0e4f;
}

struct WalkState {
  f3 t;            // distance to the next plane per axis, relative to the current step
  f3 cur;          // currentPos
  float len;       // rayLength
  uint32_t it;     // iterations of this RayMarch/RayMarchShadow call (VRT_MAX_STEPS cap)
  uint32_t ties;   // index==3 events
  bool check_cube; // TestCube must be evaluated at the loop top
};

enum : int { WALK_MISS = 0, WALK_EVENT = 1, WALK_CAP = 2 };

// floor(x) -> int in one VALU op; x is already clamped to [0, N] by the caller
__device__ __forceinline__ uint32_t cvt_flr(float x) {
  int32_t r;
  asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
  return uint32_t(r);
}

// Max of x over the ACTIVE lanes only, as a wave-uniform value. (A __shfl reduction would also
// read inactive lanes' stale registers, e.g. a step count of a lane that already stopped at the
// cap, and stall the others.) Scalar loop: each round takes the value of an active lane holding a
// larger x (ballot covers active lanes only), so it ends after <= 64 rounds, usually one.
__device__ __forceinline__ uint32_t active_max(uint32_t x) {
  uint32_t m = __builtin_amdgcn_readfirstlane(x);
  for (;;) {
    const unsigned long long bigger = __ballot(x > m);
    if (bigger == 0ull) return m;
    m = __builtin_amdgcn_readlane(x, int(__builtin_ctzll(bigger)));
  }
}

// x + (a && b ? 1 : 0) as one v_addc with the lane mask as carry-in (active lanes only). The
// masks of a and b are taken separately (each a plain v_cmp result) and ANDed in SALU; a ballot
// of the combined bool would be materialised in a VGPR first.
__device__ __forceinline__ uint32_t add_if_both(uint32_t x, bool a, bool b) {
  const unsigned long long m = __builtin_amdgcn_ballot_w64(a) & __builtin_amdgcn_ballot_w64(b);
  unsigned long long co;
  asm("v_addc_co_u32_e64 %0, %1, %0, 0, %2" : "+v"(x), "=s"(co) : "s"(m));
  return x;
}

// crossed-axis index from the compare masks: mez ? 2 : (mey ? 1 : 0), two v_cndmask
__device__ __forceinline__ uint32_t axis_index(unsigned long long mey, unsigned long long mez) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, 0, 1, %1\n\tv_cndmask_b32_e64 %0, %0, 2, %2" : "=&v"(r) : "s"(mey), "s"(mez));
  return r;
}

// m's lane bit ? if_set : if_clear, as one v_cndmask on an SGPR lane mask
__device__ __forceinline__ float sel_mask(unsigned long long m, float if_set, float if_clear) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(m));
  return r;
}

// m's lane bit ? if_set : if_clear on 32-bit integers (one v_cndmask)
__device__ __forceinline__ uint32_t sel_mask_u(unsigned long long m, uint32_t if_set, uint32_t if_clear) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(m));
  return r;
}

// LDS loads through a 32-bit LDS byte address
typedef __attribute__((address_space(3))) const float4 lds_float4;
__device__ __forceinline__ uint32_t lds_addr(const float4* p) {
  return uint32_t(reinterpret_cast<size_t>((lds_float4*)p));
}
__device__ __forceinline__ float4 lds_load(uint32_t addr) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const v4f lds_v4f;
  const v4f r = *(lds_v4f*)(size_t)addr;
  return make_float4(r.x, r.y, r.z, r.w);
}

// keep a per-ray constant in a register (stops the compiler re-deriving it inside the loop: the
// IEEE 1/d per DDA step instead of a register read; v2 of DESIGN.md §6's performance log)
__device__ __forceinline__ float opaque(float x) {
  asm volatile("" : "+v"(x));
  return x;
}

// The DDA loop of RayMarch / RayMarchShadow (voxel.glsl:273-298, :317-382) up to the first event.
// Event: SHADOW -> an opaque voxel (HasVoxel && !transparent); otherwise the sampled byte differs
// from the ray's medium, which covers both the hit (:353) and the leave-transparent case (:357).
// Every float op of a step is the reference's, in its order; only their scheduling differs:
//  - the inner loop exits on a cheap superset of the stop conditions (a sample outside the
//    volume, a byte != medium, the length, the cap); the outer loop then replays the reference's
//    decisions exactly: the event of that iteration, else the next iteration's loop-top tests
//    (length, TestCube — which can only fail after an outside sample — and the cap), and
//    re-enters the inner loop when none fires;
//  - the t update of a step (independent of the voxel) is issued before the voxel-load wait and
//    is simply dead after an event.
template <bool SHADOW, bool EXACT>
__device__ __forceinline__ int dda_walk(const Ctx& c, const f3 pos, const f3 dir, const f3 rcp,
                                        float len0, uint32_t medium, WalkState& w, int& axis_out,
                                        int32_t& vidx_out, uint32_t& v_out) {
  const f3 step = sign3(dir);
  const f3 hs = mk(0.5f * step.x, 0.5f * step.y, 0.5f * step.z);
  f3 t = w.t, cur = w.cur;
  float len = w.len;
  uint32_t it = w.it, ties = w.ties;
  bool check = w.check_cube;
  int result;
  for (;;) {
    // loop-top tests of the reference, in its order: length, TestCube, then our step cap
    if (!(len < c.max_len) || (check && !test_cube(cur, dir, c.fn))) {
      result = WALK_MISS;
      break;
    }
    if (it >= VRT_MAX_STEPS) {
      result = WALK_CAP;
      break;
    }
    // inner loop; live-outs kept in VGPRs (a bool live out of a divergent loop costs SALU mask
    // merges every iteration): the pre-update t (-> crossed axis), the texel coordinates, the raw
    // byte, and pidx_sel = the padded index, or ~0 for an outside sample
    f3 tp;
    uint32_t vi, vj, vk, v_raw, pidx_sel;
    // step counter of this inner loop: wave-uniform (every active lane enters together), so it
    // lives in an SGPR; its bound keeps every lane's total <= VRT_MAX_STEPS, the exact per-lane
    // cap is the outer test above
    const uint32_t k_max = VRT_MAX_STEPS - active_max(it);
    const uint32_t it0 = it;
    uint32_t k = 0;
    for (;;) {
      ++k;
      float tmin;
      if (EXACT) tmin = gmin(t.x, gmin(t.y, t.z));
      else tmin = __builtin_fminf(t.x, __builtin_fminf(t.y, t.z));
      tp = mk(t.x - tmin, t.y - tmin, t.z - tmin);
      len += tmin;
      const float s = len - len0;
      cur = mk(pos.x + s * dir.x, pos.y + s * dir.y, pos.z + s * dir.z);
      const bool ex = tp.x == 0.0f, ey = tp.y == 0.0f, ez = tp.z == 0.0f;
      f3 smp;
      if (EXACT) {
        smp = mk(cur.x + (0.5f * float(ex)) * step.x, cur.y + (0.5f * float(ey)) * step.y,
                 cur.z + (0.5f * float(ez)) * step.z);
      } else {  // same voxel: the +-0 added on an un-crossed axis only flips the sign of a zero
        smp = mk(cur.x + (ex ? hs.x : 0.0f), cur.y + (ey ? hs.y : 0.0f), cur.z + (ez ? hs.z : 0.0f));
      }
      // branch-free fetch: clamp to [0,N] (med3; NaN -> in range), floor; the sample is inside
      // iff clamping left it unchanged (NaN: outside); GL_REPEAT's N -> 0 is in the layout
      const float qx = __builtin_amdgcn_fmed3f(smp.x, 0.0f, c.fn);
      const float qy = __builtin_amdgcn_fmed3f(smp.y, 0.0f, c.fn);
      const float qz = __builtin_amdgcn_fmed3f(smp.z, 0.0f, c.fn);
      const bool inb = (qx == smp.x) & (qy == smp.y) & (qz == smp.z);
      vi = cvt_flr(qx);
      vj = cvt_flr(qy);
      vk = cvt_flr(qz);
      const uint32_t pidx = mad24(mad24(vk, c.p, vj), c.p, vi);
      v_raw = load_u16(c.vox, pidx) & kVoxMask;
      if (ey & ez) ties++;  // intersectionAxis[3]: rare, a skipped branch otherwise
      // t update for the crossed axis (voxel.glsl:296/381), while the load is in flight
      const bool az = ez, ay = ey & !ez, ax = !ey & !ez;  // axis = ez ? 2 : ey ? 1 : 0
      const float pa = az ? pos.z : (ay ? pos.y : pos.x);
      const float da = az ? dir.z : (ay ? dir.y : dir.x);
      const float ca = az ? cur.z : (ay ? cur.y : cur.x);
      // sign(d) on the crossed axis; on the fast path d != 0, so it is copysign(1, d) (one v_bfi)
      const float sa = EXACT ? (az ? step.z : (ay ? step.y : step.x)) : __builtin_copysignf(1.0f, da);
      const float num = (ca + sa) - pa;
      float q;
      if (EXACT) q = num / da;
      else q = div_rn(num, da, az ? rcp.z : (ay ? rcp.y : rcp.x));
      q = q - s;
      t = mk(ax ? q : tp.x, ay ? q : tp.y, az ? q : tp.z);
      pidx_sel = inb ? pidx : ~0u;
      // materialise: no SALU live-out mask for inb (v9, DESIGN.md §6 log: 0.316 -> 0.310 ms with
      // the other live-out masks removed)
      asm volatile("" : "+v"(pidx_sel));
      const bool hit = SHADOW ? (v_raw != 0u && v_raw != 2u) : (v_raw != medium);
      if (!inb | hit | !(len < c.max_len) | (k >= k_max)) break;
    }
    it = it0 + k;
    const bool inb = pidx_sel != ~0u;
    // outside samples read 0 (GetVoxel :151-152)
    const uint32_t v = inb ? v_raw : 0u;
    const bool event = SHADOW ? (v != 0u && v != 2u) : (v != medium);
    if (event) {
      axis_out = tp.z == 0.0f ? 2 : (tp.y == 0.0f ? 1 : 0);
      vidx_out = inb ? canonical_index(c, vi, vj, vk) : -1;
      v_out = v;
      check = !inb;  // on re-entry (new direction after a refraction): re-test iff outside
      result = WALK_EVENT;
      break;
    }
    check = !inb;  // not an event: evaluate the next iteration's loop-top tests
  }
  w.t = t;
  w.cur = cur;
  w.len = len;
  w.it = it;
  w.ties = ties;
  w.check_cube = check;
  return result;
}

// ---------------------------------------------------------------- empty-space step skipping --
//
// The packed volume carries, per voxel v, a skip distance G(v) such that every voxel of a box
// B(v) is empty and inside the volume, where B(v) reaches G voxels ahead of v along the ray's
// direction on every axis (faces (v + c0) + sgn*G, c0 = 0 / 1 for d > 0 / < 0) and at least one
// voxel behind v:
//  - octant layout (N <= 512; 8 volumes, one per direction octant, step s = sign(d)):
//    G(v) = F(v - s) - 1, F(u) = edge of the largest empty in-volume cube anchored at u and
//    extending along s, so B(v) = [v - s, v + (G - 1) s] (capped at kFwdCap - 1). Looking only
//    ahead, it is far larger than the centred distance behind surfaces: shadow rays leaving the
//    ground and rays moving away from geometry skip up to ~4x fewer sampled steps
//    (scripts/skipsim.py);
//  - single layout (N = 1024, where 8 volumes would overflow 32-bit offsets): G = D, the
//    centred Chebyshev distance to the nearest non-empty voxel or the outside (capped at
//    kDistCap), B(v) = [v - D + 1, v + D - 1]^3.
// Why one voxel behind: on an axis crossed at the sampled step, currentPos = pos + s*dir may round
// to just short of the crossed plane, and a later step that crosses another axis within that
// rounding distance samples floor(currentPos) there, i.e. the voxel behind v on that axis.
// After a sampled step whose texel is empty with G >= 2, an air ray (or a shadow ray) computes
// s_lim, the ray parameter up to which its position provably stays inside B(v) (forward faces
// pulled in by kSkipMargin, far above the float error of cur = pos + s*dir; positions only move
// forward, so the back faces need no test). A step with s < s_lim therefore samples an empty voxel
// inside the volume — no event, no TestCube — and needs only the exact DDA state update; the
// sample, its address and the load are skipped. Every float op that defines the walk's state is
// still executed, in the reference's order, so the walk is bit-identical.
constexpr uint32_t kDistCap = 64;  // (profiles/r01_v32_ab_distance_cap.log: 128/255 add nothing)
static_assert(kDistCap >= 2 && kDistCap <= 255, "D is stored in 8 bits");
#if defined(VRT_FWD_CAP) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_FWD_CAP is an A/B knob of make variant builds"
#endif
#ifndef VRT_FWD_CAP
#define VRT_FWD_CAP 128
#endif
constexpr uint32_t kFwdCap = VRT_FWD_CAP;  // cap of F (G = F - 1 in 8 bits): 128 vs 64 C4 -1.4 %, C1-C3 +-0.3 % (r03_s42)
static_assert(kFwdCap >= 3 && kFwdCap <= 255, "F and G are stored in 8 bits");
constexpr float kSkipMargin = 1.0f / 256.0f;

// LEN0Z: the caller guarantees len0 == +0 (the primary ray, voxel.glsl:430), so
// s = rayLength - ray.rayLength is rayLength itself (x - (+0) == x): one VALU less per step.
// s_init > 0: a first skip window [0, s_init) known from a certified walk of the same ray
// (CertResult::us: every crossing before it settled, each in the volume and not an event), so
// those steps replay only the state update; else the first step samples.
template <bool SHADOW, bool STATS, bool LEN0Z = false>
__device__ __forceinline__ int skip_walk(const Ctx& c, const f3 pos, const f3 dir, const f3 rcp,
                                         float len0, uint32_t medium, WalkState& w, int& axis_out,
                                         int32_t& vidx_out, uint32_t& v_out, float s_init = -1.0f) {
  // fast path: every dir component is non-zero, so sign(d) = copysign(1, d)
  const f3 step = mk(__builtin_copysignf(1.0f, dir.x), __builtin_copysignf(1.0f, dir.y),
                     __builtin_copysignf(1.0f, dir.z));
  const f3 hs = mk(0.5f * step.x, 0.5f * step.y, 0.5f * step.z);
  // skip-box face in travel direction: B = (v + c0) + sgn * (D - margin); c0 = 0 / 1 for d > 0 / < 0
  const f3 c0 = mk(dir.x > 0.0f ? 0.0f : 1.0f, dir.y > 0.0f ? 0.0f : 1.0f, dir.z > 0.0f ? 0.0f : 1.0f);
  const f3 boff = mk((c0.x - pos.x) * rcp.x, (c0.y - pos.y) * rcp.y, (c0.z - pos.z) * rcp.z);
  // the crossed axis' operands per step from this lane's LDS table
  c.ax[0] = make_float4(pos.x, dir.x, rcp.x, step.x);
  c.ax[kAxStride] = make_float4(pos.y, dir.y, rcp.y, step.y);
  c.ax[2 * kAxStride] = make_float4(pos.z, dir.z, rcp.z, step.z);
  uint32_t ax_a0 = lds_addr(c.ax), ax_a1 = ax_a0 + 16u * kAxStride, ax_a2 = ax_a0 + 32u * kAxStride;
  // three VGPRs, not re-derived per step (v34: C4 -2.9 %, C2 -2.7 %,
  // profiles/r01_v34_ab_lds_address_select.log)
  asm volatile("" : "+v"(ax_a0), "+v"(ax_a1), "+v"(ax_a2));
  const bool skip_ok = SHADOW || medium == 0u;
  // this ray's octant volume (its skip distances look along the ray's direction); uniform for
  // shadow rays. Every octant volume holds the same voxel bytes.
  const uint32_t obase =
      ((dir.x < 0.0f ? 1u : 0u) | (dir.y < 0.0f ? 2u : 0u) | (dir.z < 0.0f ? 4u : 0u)) * c.ostride;
  // Skip windows also end where the length test could first fail: s = fl(len - len0) is
  // monotone in len, so s < fl(max_len - len0) implies len < max_len (NaN: no window at all).
  const float s_len = LEN0Z ? c.max_len : c.max_len - len0;
  float s_first = VRT_PREFIX && s_init > 0.0f ? __builtin_fminf(s_init, s_len) : -1.0f;
  f3 t = w.t;
  float len = w.len;
  uint32_t it = w.it, ties = w.ties;
  bool check = w.check_cube;
  int result;
  constexpr uint32_t kOutside = 0x100u;
  for (;;) {
    // loop-top tests of the reference, in its order: length, TestCube, then our step cap.
    // check is only set after an outside sample; currentPos is that step's (len unchanged since),
    // recomputed with the same two ops rather than carried through the step loop
    if (!(len < c.max_len)) {
      result = WALK_MISS;
      break;
    }
    if (check) {
      const float sc = LEN0Z ? len : len - len0;
      if (!test_cube(mk(pos.x + sc * dir.x, pos.y + sc * dir.y, pos.z + sc * dir.z), dir, c.fn)) {
        result = WALK_MISS;
        break;
      }
    }
    if (it >= VRT_MAX_STEPS) {
      result = WALK_CAP;
      break;
    }
    const uint32_t k_max = VRT_MAX_STEPS - active_max(it);
    const uint32_t it0 = it;
    uint32_t k = 0;
    // this lane's step count at its exit: set by the stopping (sampled) step; lanes that run
    // into the uniform bound leave with k == k_max. Keeps k from being copied to a VGPR per step.
    uint32_t k_exit = k_max;
    // recorded by the stopping (sampled) step only; lanes that leave on the bound: no event
    uint32_t x_v = SHADOW ? 0u : medium, x_axis = 0u, x_out = 0u;  // x_out: sample was outside
    int32_t x_vidx = -1;
    float s_lim = s_first;  // no skip window yet (-1: the first step samples), or the certified prefix
    s_first = -1.0f;
    for (;;) {
      if (k >= k_max) break;  // wave-uniform step bound (scalar branch)
      ++k;
      const float tmin = __builtin_fminf(t.x, __builtin_fminf(t.y, t.z));
      const f3 tp = mk(t.x - tmin, t.y - tmin, t.z - tmin);
      len += tmin;
      const float s = LEN0Z ? len : len - len0;
      const bool ey = tp.y == 0.0f, ez = tp.z == 0.0f;
      if (STATS) ties = add_if_both(ties, ey, ez);  // intersectionAxis[3] (counter/flag only)
      // t update for the crossed axis (voxel.glsl:296/381)
      // crossed axis: z if ez (index 2, and 3 clamped), else y if ey, else x. Selected with the
      // compare masks kept in SGPRs (the compiler re-derives !ez with another v_cmp otherwise).
      const unsigned long long mey = __builtin_amdgcn_ballot_w64(ey);
      const unsigned long long mez = __builtin_amdgcn_ballot_w64(ez);
      // the crossed axis' entry address straight from the masks: two v_cndmask, no index math
      const float4 ae = lds_load(sel_mask_u(mez, ax_a2, sel_mask_u(mey, ax_a1, ax_a0)));
      const float pa = ae.x, da = ae.y, ra = ae.z, sa = ae.w;
      const float ca = pa + s * da;  // == cur on that axis: the same two ops
      const float num = (ca + sa) - pa;
      const float q = div_rn(num, da, ra) - s;
      t = mk(sel_mask(mey | mez, tp.x, q), sel_mask(mey & ~mez, q, tp.y), sel_mask(mez, q, tp.z));
      // issue the t update before the sample's load wait (v2: its ALU then overlaps the load)
      asm volatile("" :: "v"(t.x), "v"(t.y), "v"(t.z));
      if (!(s < s_lim)) {  // a sampled step (GetVoxel, voxel.glsl:149-154)
        const f3 cur = mk(pos.x + s * dir.x, pos.y + s * dir.y, pos.z + s * dir.z);
        const bool ex = tp.x == 0.0f;
        const f3 smp = mk(cur.x + (ex ? hs.x : 0.0f), cur.y + (ey ? hs.y : 0.0f),
                          cur.z + (ez ? hs.z : 0.0f));
        const float qx = __builtin_amdgcn_fmed3f(smp.x, 0.0f, c.fn);
        const float qy = __builtin_amdgcn_fmed3f(smp.y, 0.0f, c.fn);
        const float qz = __builtin_amdgcn_fmed3f(smp.z, 0.0f, c.fn);
        const bool inb = (qx == smp.x) & (qy == smp.y) & (qz == smp.z);
        const uint32_t vi = cvt_flr(qx), vj = cvt_flr(qy), vk = cvt_flr(qz);
        const uint32_t pidx = mad24(mad24(vk, c.p, vj), c.p, vi);
        const uint32_t packed = load_u16_at(c.vox, pidx, obase);
        const uint32_t v_raw = packed & kVoxMask;
        const uint32_t dist = packed >> kDistShift;
        const uint32_t v_ev = inb ? v_raw : kOutside;
        // exit parameter of the pulled-in box face per axis, ((v + c0) + sgn*fd - pos) * rcp,
        // as v*rcp + (fd*|rcp| + boff): only has to be conservative (error <~ 4e-4 |rcp| for
        // N <= 1024, against the 1/256 * |rcp| face margin), so it may contract
        const float fd = float(dist) - kSkipMargin;
        const float lx = __builtin_fmaf(float(vi), rcp.x, __builtin_fmaf(fd, __builtin_fabsf(rcp.x), boff.x));
        const float ly = __builtin_fmaf(float(vj), rcp.y, __builtin_fmaf(fd, __builtin_fabsf(rcp.y), boff.y));
        const float lz = __builtin_fmaf(float(vk), rcp.z, __builtin_fmaf(fd, __builtin_fabsf(rcp.z), boff.z));
        const bool open = skip_ok & inb & (v_raw == 0u) & (dist >= 2u);
        s_lim = open ? __builtin_fminf(__builtin_fminf(lx, ly), __builtin_fminf(lz, s_len)) : -1.0f;
        // stop the inner loop on: outside sample, a byte that is an event, the length. Only a
        // sampled step can stop it: a skipped one reads an empty in-volume texel and has
        // s < s_len, hence len < max_len (see s_len).
        const bool stop = SHADOW ? ((v_ev & ~2u) != 0u) : (v_ev != medium);
        if (stop | !(len < c.max_len)) {
          k_exit = k;
          x_v = inb ? v_raw : 0u;  // outside samples read 0 (GetVoxel :151-152)
          x_out = inb ? 0u : 1u;
          x_axis = axis_index(mey, mez);
          x_vidx = inb ? int32_t(canonical_index(c, vi, vj, vk)) : -1;
          // integers in VGPRs: a bool carried out of a divergent loop costs SALU mask merges
          // (v28 register-lean walk: 0.2146 -> 0.2038 ms with 8 waves, DESIGN.md §6 log)
          asm volatile("" : "+v"(k_exit), "+v"(x_v), "+v"(x_axis), "+v"(x_vidx), "+v"(x_out));
          break;
        }
      }
    }
    it = it0 + k_exit;
    const bool event = SHADOW ? (x_v != 0u && x_v != 2u) : (x_v != medium);
    asm volatile("" : "+v"(x_out));  // (v28, as above: kept in a VGPR across the exit)
    check = x_out != 0u;
    if (event) {  // events only come from sampled steps
      axis_out = int(x_axis);
      vidx_out = x_vidx;
      v_out = x_v;
      result = WALK_EVENT;
      break;
    }
  }
  const float s_end = LEN0Z ? len : len - len0;  // currentPos of the last step (the hit point on an event)
  w.t = t;
  w.cur = mk(pos.x + s_end * dir.x, pos.y + s_end * dir.y, pos.z + s_end * dir.z);
  w.len = len;
  w.it = it;
  w.ties = ties;
  w.check_cube = check;
  return result;
}

// RayMarch walk: per-ray reciprocals (RN(1/d), kept opaque so they stay loop-invariant).
// (The len0 == 0 specialisation of skip_walk measured neutral: r01_v37_ab_axis_major_len0_cmpt;
// round 4's pipelined, speculative, register-select and prefetching walks all measured slower
// for the exact pass's sparse batches and were removed: DESIGN.md §6, git history before r05.)
template <bool STATS>
__device__ __forceinline__ int walk_ray(const Ctx& c, const f3 pos, const f3 dir, float len0,
                                        uint32_t medium, WalkState& w, int& axis, int32_t& vidx,
                                        uint32_t& v, float s_init = -1.0f) {
  if (__builtin_expect(fast_path_ok(dir), 1)) {
    // (fast_path_ok: every |d| in [2^-64, 1e4], so rcp_newton is RN(1/d))
    const f3 rcp = mk(opaque(rcp_newton(dir.x)), opaque(rcp_newton(dir.y)), opaque(rcp_newton(dir.z)));
    return skip_walk<false, STATS>(c, pos, dir, rcp, len0, medium, w, axis, vidx, v, s_init);
  }
  return dda_walk<false, true>(c, pos, dir, dir, len0, medium, w, axis, vidx, v);
}

// RayMarchShadow walk: the direction is normalize(u_SunDir) for every ray (uniform constants)
template <bool STATS>
__device__ __forceinline__ int walk_shadow(const Ctx& c, const f3 pos, float len0, WalkState& w) {
  int axis;
  int32_t vidx;
  uint32_t v;
  if (__builtin_expect(fast_path_ok(c.sun_n), 1))
    return skip_walk<true, STATS>(c, pos, c.sun_n, c.sun_rcp, len0, 0u, w, axis, vidx, v);
  return dda_walk<true, true>(c, pos, c.sun_n, c.sun_n, len0, 0u, w, axis, vidx, v);
}

// GetReflectionRay (voxel.glsl:203-215)
// GetColor (:174-182). Textured: GetTextureCoordinate (:167-172) on the hit's face plane
// intersectionAxis[axis][1..2] (:93), then texture(u_TextureUnit, uv): NEAREST + REPEAT,
// i = floor(u * S) mod S (GL 4.5 §8.14.2; NaN -> 0 via v_cvt_flr), texels b / 255.
template <bool TEX>
__device__ __forceinline__ float4 get_color(const Ctx& c, const Hit& h) {
  const uint32_t m = mat_id(h.voxel);
  if (!TEX) return mat_color(m);
  const float px = h.axis == 0 ? h.point.z : h.point.x;   // intersectionAxis[a][1]
  const float py = h.axis == 2 ? h.point.y : (h.axis == 1 ? h.point.z : h.point.y);  // [a][2]
  const float fx = px - floorf(px), fy = py - floorf(py);
  const float tx = ((fx + float(mat_tex_x(m))) * c.atlas_fts) / c.atlas_fs;
  const float ty = (((1.0f - fy) + float(mat_tex_y(m))) * c.atlas_fts) / c.atlas_fs;
  const float u = tx, v = 1.0f - ty;
  const uint32_t i = cvt_flr(u * c.atlas_fs) & c.atlas_mask;
  const uint32_t j = cvt_flr(v * c.atlas_fs) & c.atlas_mask;
  const uint32_t t = c.atlas[j * (c.atlas_mask + 1u) + i];
  return make_float4(float(t & 0xFFu) / 255.0f, float((t >> 8) & 0xFFu) / 255.0f,
                     float((t >> 16) & 0xFFu) / 255.0f, float(t >> 24) / 255.0f);
}

__device__ __forceinline__ Ray reflection_ray(const Ctx& c, const Ray& ray, const Hit& h) {
  Ray r;
  r.voxel = 0;
  r.pos = h.point;
  r.dir = randomize(reflect3(ray.dir, h.normal), h.point, c.refl_noise, c.time);
  r.len = h.len;
  r.energy = ray.energy * (1.0f - dot3(mk(-h.normal.x, -h.normal.y, -h.normal.z), ray.dir));
  r.rdepth = ray.rdepth + 1;
  r.tdepth = ray.tdepth;
  return r;
}

// GetRefractionRay (voxel.glsl:217-246)
template <bool TEX>
__device__ __forceinline__ Ray refraction_ray(const Ctx& c, const Ray& ray, const Hit& h, Counters& k) {
  const uint32_t outv = get_voxel(c, h.point + h.normal * 0.5f);
  const uint32_t inv = get_voxel(c, h.point - h.normal * 0.5f);
  k.c[VRT_CNT_REFRACTION_PROBES]++;
  const float eta = mat_refr(outv) / mat_refr(inv);
  Ray r;
  r.voxel = h.voxel;
  r.pos = h.point;
  r.dir = refract3(normalize3(ray.dir), h.normal, eta);
  if (r.dir.x == 0.0f && r.dir.y == 0.0f && r.dir.z == 0.0f) {  // total internal reflection
    r = reflection_ray(c, ray, h);
    r.voxel = ray.voxel;
    r.energy = ray.energy;
  } else {
    r.dir = randomize(r.dir, r.pos, c.refr_noise, c.time);
    r.energy = ray.energy;
    if (ray.voxel == 0) r.energy *= 1.0f - get_color<TEX>(c, h).w;  // :239-240
  }
  r.len = h.len;
  r.rdepth = ray.rdepth;
  r.tdepth = ray.tdepth + 1;
  return r;
}

__device__ __forceinline__ void walk_init(WalkState& w, const Ray& ray) {
  w.len = ray.len;
  w.cur = ray.pos;
  w.t = initial_t(ray.dir, ray.pos, ray.pos);
  w.it = 0;
  w.ties = 0;
  w.check_cube = true;
}

__device__ __forceinline__ void walk_account(const WalkState& w, int r, int steps_slot,
                                             Counters& k, uint32_t& steps, uint32_t& flags) {
  steps += w.it;
  k.c[steps_slot] += w.it;
  k.c[VRT_CNT_TIE3] += w.ties;
  if (w.ties) flags |= VRT_HIT_FLAG_TIE3;
  if (r == WALK_CAP) {
    k.c[VRT_CNT_STEP_CAP]++;
    flags |= VRT_HIT_FLAG_STEP_CAP;
  }
}

// RayMarchShadow (voxel.glsl:259-300): true when an opaque voxel blocks the sun.
template <bool STATS>
__device__ __forceinline__ bool march_shadow(const Ctx& c, const Ray& ray, Counters& k, uint32_t& steps,
                             uint32_t& flags) {
  WalkState w;
  walk_init(w, ray);
  const int r = walk_shadow<STATS>(c, ray.pos, ray.len, w);
  walk_account(w, r, VRT_CNT_SHADOW_STEPS, k, steps, flags);
  return r == WALK_EVENT;
}

// RayMarch (voxel.glsl:302-384); `ray` is inout (in-volume refraction rewrites it, :361)
// PRIMARY: the primary ray (len 0, medium air: every event is a hit, no in-volume refraction)
// s_init (PRIMARY only): the certified prefix of the primary walk (skip_walk)
template <bool STATS, bool TEX, bool PRIMARY = false>
__device__ __forceinline__ Hit march(const Ctx& c, Ray& ray, Counters& k, uint32_t& steps, uint32_t& flags,
                     float s_init = -1.0f) {
  Hit h;
  h.found = false;
  h.vidx = -1;
  h.len = 0.0f;
  h.voxel = 0;
  h.point = mk(0.0f, 0.0f, 0.0f);
  h.normal = h.point;
  h.axis = 0;
  WalkState w;
  walk_init(w, ray);
  uint32_t medium = ray.voxel;
  int internal = 0;
  int r;
  for (;;) {
    int axis;
    int32_t vidx;
    uint32_t v;
    r = walk_ray<STATS>(c, ray.pos, ray.dir, ray.len, PRIMARY ? 0u : medium, w, axis, vidx, v,
                        PRIMARY ? s_init : -1.0f);
    if (r != WALK_EVENT) break;
    f3 normal = mk(0.0f, 0.0f, 0.0f);
    set_comp(normal, axis, -gsign(comp(ray.dir, axis)));
    // HasVoxel(voxel) && voxel != rayVoxel (:353); a primary ray's medium is air, so its
    // every event is a hit
    if (PRIMARY || v != 0u) {
      h.found = true;
      h.voxel = v;
      h.vidx = vidx;
      h.point = w.cur;
      h.len = w.len;
      h.normal = normal;
      h.axis = axis;
      break;
    }
    // rayVoxel != 0 && voxel == 0: leaving a transparent voxel, refract in place (:357-380)
    Hit e;
    e.found = true;
    e.voxel = 0;
    e.vidx = vidx;
    e.point = w.cur;
    e.len = w.len;
    e.normal = normal;
    e.axis = axis;
    const f3 old_dir = ray.dir;
    ray = refraction_ray<TEX>(c, ray, e, k);
    ray.tdepth--;
    if (ray.voxel == medium) {
      internal++;
      if (internal > 10) {
        ray.dir = old_dir;
        ray.voxel = 0;
      }
    }
    medium = ray.voxel;
    w.t = initial_t(ray.dir, w.cur, ray.pos);
    const f3 step = sign3(ray.dir);
    const float q = ((comp(w.cur, axis) + comp(step, axis)) - comp(ray.pos, axis)) /
                        comp(ray.dir, axis) - (w.len - ray.len);
    set_comp(w.t, axis, q);
  }
  walk_account(w, r, VRT_CNT_DDA_STEPS, k, steps, flags);
  return h;
}

// Brightness of a hit that is not in shadow (voxel.glsl:405-409)
template <bool TEX>
__device__ __forceinline__ float lit_brightness(const Hit& h, const f3 sun_dir, const f3 ray_dir) {
  const uint32_t m = mat_id(h.voxel);
  const float diffuse = mat_kd(m) * gmax(dot3(h.normal, sun_dir), 0.0f);
  const float specular =
      mat_ks(m, TEX) * gpow(gmax(dot3(reflect3(sun_dir, h.normal), ray_dir), 0.0f), mat_exp(m, TEX));
  return kAmbient + diffuse + specular;
}

// RayColor (:184-188)
template <bool TEX>
__device__ __forceinline__ void apply_hit_color(const Ctx& c, const Hit& h, float energy,
                                                float brightness, f3& color) {
  const float4 col = get_color<TEX>(c, h);
  color.x = mixf(color.x, col.x * col.w * brightness, energy);
  color.y = mixf(color.y, col.y * col.w * brightness, energy);
  color.z = mixf(color.z, col.z * col.w * brightness, energy);
}

// GetSkyboxColor (:386-393), then the second mix at :420
__device__ __forceinline__ void apply_sky_color(const Ctx& c, const Ray& ray, f3& color) {
  const f3 u = normalize3(ray.dir);
  const float sun = 10.0f * gpow(dot3(c.sun_n, u), 400.0f);
  const float grad = (u.y + 1.0f) * 0.5f;
  const float sy = c.sky_sy;  // gmax(u_SunDir.y, 0), precomputed (a wave-uniform constant)
  const f3 sk = mk(gmax(0.0f, sun) * sy, gmax(grad * 0.75f, sun) * sy, gmax(grad, 0.0f) * sy);
  const float a1 = 1.0f - ray.energy;
  const f3 s1 = mk(mixf(sk.x, color.x, a1), mixf(sk.y, color.y, a1), mixf(sk.z, color.z, a1));
  color = mk(mixf(s1.x, color.x, a1), mixf(s1.y, color.y, a1), mixf(s1.z, color.z, a1));
}

__device__ __forceinline__ int cert_shadow_exact(const Ctx& c, const Hit& h);

// TraceWithShadow's colour update (voxel.glsl:395-423) for the exact march's result h. CSH
// (stats-free colour-only): the shadow bit by a certified walk from the exact hit point when it
// settles it (cert_shadow_exact), and no shadow walk when it cannot change the brightness
// (lit == ambient).
template <bool STATS, bool TEX, bool CSH>
__device__ __forceinline__ void shade(const Ctx& c, const Ray& ray, const Hit& h, f3& color, Counters& k,
                                      uint32_t& steps, uint32_t& flags) {
  static_assert(!CSH || !STATS, "certified shadows in stats-free instances only");
  if (h.found) {
    Ray sr;  // GetShadowRay (:191-201)
    sr.voxel = h.voxel;
    sr.pos = h.point;
    sr.dir = c.sun_n;
    sr.len = h.len;
    sr.energy = ray.energy;
    sr.rdepth = 0;
    sr.tdepth = 0;
    float brightness;
    if (CSH) {
      const float lit = lit_brightness<TEX>(h, c.sun_n, ray.dir);
      int blocked = 0;
      if (lit != kAmbient && !shadow_free_hit(h.voxel, TEX)) {
        blocked = cert_shadow_exact(c, h);
        if (blocked < 0) blocked = march_shadow<STATS>(c, sr, k, steps, flags) ? 1 : 0;
      }
      brightness = blocked ? kAmbient : lit;
    } else {
      k.c[VRT_CNT_SHADOW_RAYS]++;
      const bool in_shadow = march_shadow<STATS>(c, sr, k, steps, flags);
      brightness = in_shadow ? kAmbient : lit_brightness<TEX>(h, sr.dir, ray.dir);
    }
    apply_hit_color<TEX>(c, h, ray.energy, brightness, color);
  } else {
    apply_sky_color(c, ray, color);
  }
}

// TraceWithShadow (voxel.glsl:395-423) and the colour update it performs
template <bool STATS, bool TEX, bool PRIMARY = false, bool CSH = false>
__device__ __forceinline__ Hit trace_with_shadow(const Ctx& c, Ray& ray, f3& color, Counters& k,
                                                 uint32_t& steps, uint32_t& flags, float s_init = -1.0f) {
  const Hit h = march<STATS, TEX, PRIMARY>(c, ray, k, steps, flags, s_init);
  shade<STATS, TEX, CSH>(c, ray, h, color, k, steps, flags);
  return h;
}

// ------------------------------------------------------------ certified walks (stats-free) --
//
// The colour-only image depends on a primary walk only through its outcome — miss, or the first
// event's byte and face axis — and on a shadow walk only through blocked / not blocked
// (voxel.glsl:395-423: no hit point, length or texel index enters the colour of a non-glass hit;
// the sky colour depends on the direction alone). The exact walk (skip_walk) replays every DDA
// step's float state to be bit-identical; the CERTIFIED walk below instead follows the real ray
// with a float DDA that jumps through the empty boxes of the octant distance field, and returns
// the exact walk's outcome only when no rounding of the exact walk can change it:
//  - the exact walk's parameter at any plane crossing differs from the real one by at most
//    gam_b(u) (`cert_gamma`): its len accumulates at most u*|d|_1 + 3 non-zero steps, each adding
//    <= 2^-24 len; each t is re-anchored from currentPos (roundings of magnitude <= N + 2, times
//    1/|d_b|) and then decremented at most K times; zero-length tie steps add no rounding;
//  - crossings of two axes closer than gam_a + gam_b may come in either order or as a tie: the
//    cells the exact walk could sample instead (`alternatives`) must be non-events, else UNSURE;
//  - an event cell is a certified hit only if its entry crossing is isolated (the exact walk
//    then enters it across the same face, index = that axis) and the length test cannot stop
//    the walk first; a walk that leaves the volume or whose previous crossing lies beyond the
//    length budget (by more than the bound) is a certified miss;
//  - cells with an index N are outside on the path (the exact walk reads the GL_REPEAT plane N
//    only at a coordinate exactly N, i.e. at a near-edge crossing, where the alternatives read
//    the padded layout's plane N).
// UNSURE rays (~0.2 % of pixels at the BASELINE configs, scripts/certsim.py) and every pixel
// whose primary hit is glass (its secondary rays start at the exact hit point) take the exact
// path. Only the stats-free colour-only instance uses it: hit records and counters need the
// exact walk, and textured shading reads the hit point.

// Bounce stacks run at raised wave priority (s_setprio): they are a frame's longest waves
// (-2 % at C3, profiles/r01_v45_ab_wave_priority.log).
constexpr int kStackPrio = 3;
#ifdef VRT_CERT_DIAG  // diagnostic build only (scripts/cert_diag.py): outcome counts per pixel
__device__ unsigned long long g_cert_diag[32];
#define CERT_DIAG(i) atomicAdd(&g_cert_diag[i], 1ull)
__device__ __forceinline__ void cert_diag_iters(int slot, int it) {
  atomicAdd(&g_cert_diag[slot], (unsigned long long)it);
  int m = it;
  for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off, 64));
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  if (l == 0) atomicAdd(&g_cert_diag[slot + 2], (unsigned long long)m);
}
#else
#define CERT_DIAG(i) ((void)0)
#endif
enum : int { CERT_MISS = 0, CERT_HIT = 1, CERT_UNSURE = 2 };
constexpr float kCertMargin = 1.0f / 64.0f;  // jump boxes' forward faces pulled in (position)
constexpr int kCertMaxIter = 1024;
constexpr float kCertMaxOrigin = 4e-3f;  // parameter uncertainty of a secondary start beyond which: unsure

struct CertResult {
  int res;
  uint32_t byte;
  int axis;
  int cx, cy, cz;  // hit cell
  float u;         // crossing parameter of the hit
  float eu;        // bound of the exact walk's parameter error there
  // every step of the exact walk with parameter s < us samples an in-volume cell that is not an
  // event (the certified crossings before the last one the walk settled); 0: none known
  float us;
#ifdef VRT_CERT_DIAG
  int iters;
#endif
};

__device__ __forceinline__ uint32_t cell_texel(const Ctx& c, int i, int j, int k, uint32_t obase) {
  return load_u16_at(c.vox, mad24(mad24(uint32_t(k), c.p, uint32_t(j)), c.p, uint32_t(i)), obase);
}
// texel of a cell on the certified path: cells outside [0, N)^3 read 0 (empty, G = 0)
__device__ __forceinline__ uint32_t path_texel(const Ctx& c, int i, int j, int k, uint32_t obase) {
  const uint32_t n = uint32_t(c.n);
  if (uint32_t(i) >= n || uint32_t(j) >= n || uint32_t(k) >= n) return 0u;
  return cell_texel(c, i, j, k, obase);
}
// byte of a cell the exact walk might sample at a near-edge crossing (plane N: GL_REPEAT copy)
__device__ __forceinline__ uint32_t alt_byte(const Ctx& c, int i, int j, int k, uint32_t obase) {
  const uint32_t n = uint32_t(c.n);
  if (uint32_t(i) > n || uint32_t(j) > n || uint32_t(k) > n) return 0u;
  return cell_texel(c, i, j, k, obase) & kVoxMask;
}
// an event of the exact walk: shadow rays stop at opaque bytes (not air, not glass), other rays
// at any byte other than their medium's (voxel.glsl:353, :357)
template <bool SHADOW>
__device__ __forceinline__ bool cert_event(uint32_t b, uint32_t medium) {
  return SHADOW ? (b & ~2u) != 0u : b != medium;
}

// Certified walk from P along D (every |d| in the fast-path range) with rcp ~ 1/D (a few ulp
// suffice: the walk's own rounding is inside the 4e-5 allowance of the bound), starting in cell
// (cx, cy, cz) inside the volume. U = max_len - len0: the exact walk samples the crossing at u iff
// its len before that step is < max_len. e0: parameter uncertainty of the start (a shadow origin
// is the exact primary hit point, known to +-e0 along the primary); ed: per-axis crossing-order
// uncertainty from it; len0b: bound of len0. No crossing lies behind the start, so the start
// cell's box need not cover a cell behind it: it is read from the diagonal neighbour's texel,
// G(v + s) = F(v) - 1, i.e. the box [v, v + G s].
template <bool SHADOW>
__device__ __forceinline__ CertResult cert_walk(const Ctx& c, const f3 P, const f3 D, const f3 rcp, const float U,
                                int cx, int cy, int cz, const float e0, const f3 ed,
                                const float len0b, const uint32_t medium, const uint32_t tex0 = ~0u) {
  CertResult r;
  r.res = CERT_UNSURE;
  r.byte = 0u;
  r.axis = 0;
  r.cx = r.cy = r.cz = 0;
  r.u = 0.0f;
  r.eu = 0.0f;
  r.us = 0.0f;
  const int sx = D.x > 0.0f ? 1 : -1, sy = D.y > 0.0f ? 1 : -1, sz = D.z > 0.0f ? 1 : -1;
  const int ux = D.x > 0.0f ? 1 : 0, uy = D.y > 0.0f ? 1 : 0, uz = D.z > 0.0f ? 1 : 0;
  const f3 ar = mk(__builtin_fabsf(rcp.x), __builtin_fabsf(rcp.y), __builtin_fabsf(rcp.z));
  const float l1 = __builtin_fabsf(D.x) + __builtin_fabsf(D.y) + __builtin_fabsf(D.z);
  const uint32_t obase = ((D.x < 0.0f ? 1u : 0u) | (D.y < 0.0f ? 2u : 0u) | (D.z < 0.0f ? 4u : 0u)) * c.ostride;
  // Rounding bounds as polynomials in the crossing parameter u (2x safety factor on 2^-24):
  //   K(u) = u |d|_1 + 3 non-zero exact steps, sum_k len_k <= (K + 3)^2 / (2 |d|_1) + K (len0 + 1),
  //   gam_b(u) = 2^-24 (sum len + 2 (u + len0) + (K + 3N + 8) |1/d_b|) + 4e-5 + e0 + ed_b,
  //   gL(u) = 2^-23 sum len + 1e-4 + e0 (the length test)
  constexpr float k24 = 2.0f * 0x1p-24f;
  const float q2 = 0.5f * k24 * l1;
  // 18 / |d|_1 only bounds a sum: the hardware reciprocal (<= 1 ulp) scaled up by 2^-19 stays above it
  const float lin = 6.0f + l1 * (len0b + 1.0f),
              con = (18.0f * 1.0000020f) * __builtin_amdgcn_rcpf(l1) + 3.0f * (len0b + 1.0f);
  const float nterm = 3.0f * c.fn + 11.0f;
  const f3 q1 = mk(k24 * (lin + 2.0f + ar.x * l1), k24 * (lin + 2.0f + ar.y * l1), k24 * (lin + 2.0f + ar.z * l1));
  const float c0 = k24 * (con + 2.0f * len0b) + 4e-5f + e0;
  const f3 q0 = mk(c0 + k24 * ar.x * nterm + ed.x, c0 + k24 * ar.y * nterm + ed.y, c0 + k24 * ar.z * nterm + ed.z);
  const float g2 = 2.0f * q2, g1 = 2.0f * k24 * lin, g0 = 2.0f * k24 * con + 1e-4f + e0;
  // sign-folded start and direction: Ps_b + u |d_b| = s_b (P_b + u d_b) exactly (negation is exact),
  // so a landing cell is floor(s x) ^ m, m = 0 or ~0 (ceil(x) - 1 = ~floor(-x)), without branches
  const f3 Ps = mk(ux ? P.x : -P.x, uy ? P.y : -P.y, uz ? P.z : -P.z);
  const f3 Da = mk(__builtin_fabsf(D.x), __builtin_fabsf(D.y), __builtin_fabsf(D.z));
  const int mx = ux - 1, my = uy - 1, mz = uz - 1;
  f3 sig = mk((float(cx + ux) - P.x) * rcp.x, (float(cy + uy) - P.y) * rcp.y,
              (float(cz + uz) - P.z) * rcp.z);
  // start: the unguarded box from the diagonal neighbour (G(v + s) + 1 in the guarded formula)
  // (tex0: that texel, loaded by the caller beside an earlier load; ~0u: load it here)
  uint32_t tex = (tex0 != ~0u ? tex0 : path_texel(c, cx + sx, cy + sy, cz + sz, obase)) + (1u << kDistShift);
  CTRACE(c, 100 + int(SHADOW), cx, cy, cz, P.x, P.y, P.z, U);
  CTRACE(c, 101, D.x, D.y, D.z, e0, ed.x, ed.y, ed.z);
#ifdef VRT_CERT_DIAG
  r.iters = 0;
#endif
  for (int guard = 0; guard < kCertMaxIter; ++guard) {
#ifdef VRT_CERT_DIAG
    r.iters = guard + 1;
#endif
    const float s1 = __builtin_fminf(sig.x, __builtin_fminf(sig.y, sig.z));
    const int a = sig.x == s1 ? 0 : (sig.y == s1 ? 1 : 2);
    const float uu = gmax(s1, 0.0f);
    const f3 gam = mk(__builtin_fmaf(__builtin_fmaf(q2, uu, q1.x), uu, q0.x),
                      __builtin_fmaf(__builtin_fmaf(q2, uu, q1.y), uu, q0.y),
                      __builtin_fmaf(__builtin_fmaf(q2, uu, q1.z), uu, q0.z));
    // empty-space jump: the box [v - s, v + (G - 1) s] of this cell is empty and in the volume
    // (only for rays in air: empty cells are events in a glass medium)
    const uint32_t G = tex >> kDistShift;
    if (G >= 2u && (SHADOW || medium == 0u)) {
      // the box's far face on axis b is G - 1 - margin cells beyond the plane of sig_b: its
      // parameter sig_b + (G - 1 - margin) |1/d_b| up to a few ulps, far inside the margin's
      // margin |1/d_b| (|sig_b| <= ~400 |1/d_b| in a 256^3 volume: 1e-4 |1/d_b| at 3 ulps)
      const float fg1 = float(G) - (1.0f + kCertMargin);
      const float lx = __builtin_fmaf(fg1, ar.x, sig.x);
      const float ly = __builtin_fmaf(fg1, ar.y, sig.y);
      const float lz = __builtin_fmaf(fg1, ar.z, sig.z);
      // per axis: the exact walk crosses the box face of axis b within gam_b of l_b, so its steps
      // up to min_b (l_b - gam_b) sample box cells (a common max(gam) would let one nearly
      // parallel axis, |1/d_b| huge, stop every jump: ~90 us cell-by-cell walks at C3)
      const float uj = __builtin_fminf(__builtin_fminf(lx - gam.x, ly - gam.y),
                                       __builtin_fminf(lz - gam.z, U + 2.0f));
      CTRACE(c, 102, G, s1, uj, gam.x, gam.y, gam.z, 0);
      if (uj > s1) {
        // the cell the exact walk is in there: floor(x) moving up, ceil(x) - 1 moving down
        const float x = Ps.x + uj * Da.x, y = Ps.y + uj * Da.y, z = Ps.z + uj * Da.z;
        cx = int(__builtin_floorf(x)) ^ mx;
        cy = int(__builtin_floorf(y)) ^ my;
        cz = int(__builtin_floorf(z)) ^ mz;
        sig = mk((float(cx + ux) - P.x) * rcp.x, (float(cy + uy) - P.y) * rcp.y,
                 (float(cz + uz) - P.z) * rcp.z);
        tex = path_texel(c, cx, cy, cz, obase);
        continue;
      }
    }
    // one crossing, s1 on axis a; prev = the crossing before it (the exact walk's len there)
    const f3 back = mk(sig.x - ar.x, sig.y - ar.y, sig.z - ar.z);
    const float mback = gmax(back.x, gmax(back.y, back.z));
    const float prev = gmax(mback, 0.0f);
    const float gL = __builtin_fmaf(__builtin_fmaf(g2, uu, g1), uu, g0);
    if (prev > U + gL) {
      // the length test stops the walk before this crossing, unless a tie merges it into the
      // step of the one before (that step passed the test): then the exact walk still samples it
      // (a tree ray whose y and z crossings tied at len 101.1 left the glass there, refracting,
      // before its length ended the march; its sky colour took the refracted direction)
      if (s1 - mback < 2.0f * gmax(gam.x, gmax(gam.y, gam.z))) return r;
      r.res = CERT_MISS;
      return r;
    }
    const int nx = cx + (a == 0 ? sx : 0), ny = cy + (a == 1 ? sy : 0), nz = cz + (a == 2 ? sz : 0);
    const uint32_t ntex = path_texel(c, nx, ny, nz, obase);
    const float ga = a == 0 ? gam.x : (a == 1 ? gam.y : gam.z);
    // near-edge flags per other axis: ahead (crossed within the bound after s1) / behind (before).
    // A plane behind counts down to -gam_b, not 0: a ray that starts ON a plane (a shadow or
    // secondary ray from an exact hit point on the hit face) has that plane at parameter 0 up to
    // rounding, and the exact walk's currentPos stays on it — sampling the voxel beyond it — until
    // the ray has moved half an ulp of the coordinate off it (r02 s18: a shadow ray from
    // (33.000008, 127, 37.02) sampled the panel voxel (32, 127, 37) at its first x crossing, and
    // back.y rounded to just below 0 hid that alternative from the certified walk)
    // nf bits 0-2: ahead x, y, z; 3-5: behind x, y, z. They are rare: a superset test first (the
    // second smallest sig bounds every sig_b, b != a, from below, the latest back every back_b from
    // above, and ga + max gam every ga + gam_b; rounding is monotone), the flags only if it holds.
    const float tg = ga + gmax(gam.x, gmax(gam.y, gam.z));
    // the crossings up to prev are settled (this one, at s1, may not be): an exact step at s <
    // prev - tg has its real crossing before prev (gam_b <= tg), so it samples a settled cell
    r.us = prev - tg - 1e-3f;
    uint32_t nf = 0u;
    if (__builtin_amdgcn_fmed3f(sig.x, sig.y, sig.z) - s1 < tg || s1 - mback < tg) {
      const bool ahx = a != 0 && sig.x - s1 < ga + gam.x, ahy = a != 1 && sig.y - s1 < ga + gam.y,
                 ahz = a != 2 && sig.z - s1 < ga + gam.z;
      const bool bhx = a != 0 && back.x > -gam.x && s1 - back.x < ga + gam.x;
      const bool bhy = a != 1 && back.y > -gam.y && s1 - back.y < ga + gam.y;
      const bool bhz = a != 2 && back.z > -gam.z && s1 - back.z < ga + gam.z;
      nf = uint32_t(ahx) | uint32_t(ahy) << 1 | uint32_t(ahz) << 2 | uint32_t(bhx) << 3 |
           uint32_t(bhy) << 4 | uint32_t(bhz) << 5;
    }
    const uint32_t nb = ntex & kVoxMask;
    CTRACE(c, 103, nx, ny, nz, s1, a, nf, nb);
    CTRACE(c, 104, cx, cy, cz, sig.x, sig.y, sig.z, ga);
    if (cert_event<SHADOW>(nb, medium)) {
      if (!(prev + gL < U)) return r;  // the length test might stop the walk first
      if (nf == 0u) {
        r.res = CERT_HIT;
        r.byte = nb;
        r.axis = a;
        r.cx = nx;
        r.cy = ny;
        r.cz = nz;
        r.u = s1;
        r.eu = ga;
        return r;
      }
      if (SHADOW && __builtin_popcount(nf) == 1) {
        // blocked whichever way the exact walk goes: near-behind b still samples nc (or nc - e_b
        // first); near-ahead b samples nc, or cell + e_b and then nc + e_b
        bool ok = true;
        if (nf & 7u) {
          const int bx = (nf & 1u) ? sx : 0, by = (nf & 2u) ? sy : 0, bz = (nf & 4u) ? sz : 0;
          ok = cert_event<true>(alt_byte(c, cx + bx, cy + by, cz + bz, obase), 0u) ||
               cert_event<true>(alt_byte(c, nx + bx, ny + by, nz + bz, obase), 0u);
        }
        if (ok) {
          r.res = CERT_HIT;
          r.byte = nb;
        }
      }
      return r;  // hit or unsure
    }
    if (nf) {  // cells the exact walk may sample instead of the path's: all must be non-events
      const bool ahx = nf & 1u, ahy = nf & 2u, ahz = nf & 4u, bhx = nf & 8u, bhy = nf & 16u,
                 bhz = nf & 32u;
      const int nah = int(ahx) + int(ahy) + int(ahz);
      if (__builtin_popcount(nf) >= 2) {  // near a corner: the 2x2x2 block ahead and the cells behind nc
        for (int q = 1; q < 8; ++q)
          if (cert_event<SHADOW>(alt_byte(c, cx + ((q & 1) ? sx : 0), cy + ((q & 2) ? sy : 0),
                                          cz + ((q & 4) ? sz : 0), obase), medium))
            return r;
        if ((bhx && cert_event<SHADOW>(alt_byte(c, nx - sx, ny, nz, obase), medium)) ||
            (bhy && cert_event<SHADOW>(alt_byte(c, nx, ny - sy, nz, obase), medium)) ||
            (bhz && cert_event<SHADOW>(alt_byte(c, nx, ny, nz - sz, obase), medium)))
          return r;
      } else if (nah) {  // b may be crossed first, or tie: cell + e_b, nc + e_b
        const int bx = ahx ? sx : 0, by = ahy ? sy : 0, bz = ahz ? sz : 0;
        if (cert_event<SHADOW>(alt_byte(c, cx + bx, cy + by, cz + bz, obase), medium) ||
            cert_event<SHADOW>(alt_byte(c, nx + bx, ny + by, nz + bz, obase), medium))
          return r;
      } else {  // a may have been crossed before b: nc - e_b
        if (cert_event<SHADOW>(alt_byte(c, nx - (bhx ? sx : 0), ny - (bhy ? sy : 0),
                                        nz - (bhz ? sz : 0), obase), medium))
          return r;
      }
    }
    const int na = a == 0 ? nx : (a == 1 ? ny : nz);
    const int sa = a == 0 ? sx : (a == 1 ? sy : sz);
    if (uint32_t(na) >= uint32_t(c.n)) {  // left the volume (moving away on axis a)
      r.res = CERT_MISS;
      return r;
    }
    cx = nx;
    cy = ny;
    cz = nz;
    tex = ntex;
    const float np = float(na + (sa > 0 ? 1 : 0));
    if (a == 0) sig.x = (np - P.x) * rcp.x;
    else if (a == 1) sig.y = (np - P.y) * rcp.y;
    else sig.z = (np - P.z) * rcp.z;
  }
  return r;
}

// A ray that starts at a face crossing of a certified walk (a shadow or secondary ray from a hit,
// or a walk restarted by in-volume refraction): the exact origin lies within e (parameter) of
// X = P + u D0 along the parent direction D0, so within e |D0_fa| of the face plane (axis fa),
// possibly on its far side. The exact walk starts in the same cell (cx, cy, cz) on the new
// direction's side of the plane and samples the same cells if, on every other axis, X is farther
// than its uncertainty from a plane and the new ray's first crossing of that axis comes after it
// has left the face plane's neighbourhood (lead). ed: the crossing-order uncertainty the origin
// adds to the new walk.
__device__ __forceinline__ bool cert_start(const f3 X, const f3 D0, const f3 Dn, const f3 rcpn,
                                           int fa, float e, int cx, int cy, int cz, f3& ed) {
  ed = mk(2.0f * e * __builtin_fabsf(D0.x * rcpn.x), 2.0f * e * __builtin_fabsf(D0.y * rcpn.y),
          2.0f * e * __builtin_fabsf(D0.z * rcpn.z));
  const float d0a = fa == 0 ? D0.x : (fa == 1 ? D0.y : D0.z);
  const float rna = fa == 0 ? rcpn.x : (fa == 1 ? rcpn.y : rcpn.z);
  const float lead = (e * __builtin_fabsf(d0a) + 1e-5f) * __builtin_fabsf(rna);
  const float wx = (float(cx + (Dn.x > 0.0f)) - X.x) * rcpn.x;
  const float wy = (float(cy + (Dn.y > 0.0f)) - X.y) * rcpn.y;
  const float wz = (float(cz + (Dn.z > 0.0f)) - X.z) * rcpn.z;
  const f3 fr = mk(X.x - __builtin_floorf(X.x), X.y - __builtin_floorf(X.y), X.z - __builtin_floorf(X.z));
  const f3 dm = mk(e * __builtin_fabsf(D0.x) + 2e-5f, e * __builtin_fabsf(D0.y) + 2e-5f,
                   e * __builtin_fabsf(D0.z) + 2e-5f);
  const bool okx = fa == 0 || (wx >= lead + ed.x + 1e-4f && fr.x >= dm.x && 1.0f - fr.x >= dm.x);
  const bool oky = fa == 1 || (wy >= lead + ed.y + 1e-4f && fr.y >= dm.y && 1.0f - fr.y >= dm.y);
  const bool okz = fa == 2 || (wz >= lead + ed.z + 1e-4f && fr.z >= dm.z && 1.0f - fr.z >= dm.z);
  return okx && oky && okz;
}

// The cell before a hit cell along D on its crossed axis
__device__ __forceinline__ void cell_before(const CertResult& h, const f3 D, int& x, int& y, int& z) {
  x = h.cx - (h.axis == 0 ? (D.x > 0.0f ? 1 : -1) : 0);
  y = h.cy - (h.axis == 1 ? (D.y > 0.0f ? 1 : -1) : 0);
  z = h.cz - (h.axis == 2 ? (D.z > 0.0f ? 1 : -1) : 0);
}

// A Hit record for a certified hit of `ray`: point and len approximate (within h.eu along the
// ray); only the face, voxel and (in robust positions) the probes derived from it are used
__device__ __forceinline__ Hit cert_hit_record(const Ray& ray, const CertResult& h) {
  Hit hh;
  hh.found = true;
  hh.voxel = h.byte;
  hh.axis = h.axis;
  hh.vidx = -1;
  hh.len = ray.len + h.u;
  hh.point = mk(ray.pos.x + h.u * ray.dir.x, ray.pos.y + h.u * ray.dir.y, ray.pos.z + h.u * ray.dir.z);
  hh.normal = mk(0.0f, 0.0f, 0.0f);
  set_comp(hh.normal, h.axis, -gsign(comp(ray.dir, h.axis)));
  return hh;
}

// TraceWithShadow's colour update (voxel.glsl:395-418) for a certified hit of `ray`: the shadow
// bit by a certified shadow walk from the hit, unless it cannot change the brightness (lit ==
// ambient). false: unsure (colour untouched).
template <bool TEX = false>
__device__ __forceinline__ bool cert_shade_hit(const Ctx& c, const Ray& ray, const CertResult& h,
                                               const Hit& hh, f3& color, float4 col = float4()) {
  const float lit = lit_brightness<TEX>(hh, c.sun_n, ray.dir);
  float brightness = kAmbient;
  if (lit != kAmbient && !shadow_free_hit(h.byte, TEX) && VRT_DIAG_PHASE > 3) {  // otherwise the brightness is the ambient term (or irrelevant)
    const f3 S = c.sun_n;
    if (!(dot3(hh.normal, S) > 0.0f) || !fast_path_ok(S)) { CERT_DIAG(5); return false; }  // back face
    // shadow origin: the exact hit point; start cell: the air cell in front of the hit face
    int ax, ay, az;
    cell_before(h, ray.dir, ax, ay, az);
    // the shadow walk's start texel (the diagonal neighbour in the sun's octant volume) is loaded
    // first, so its latency overlaps the start checks and the air-cell load (same octant volume:
    // every octant volume holds the same voxel bytes)
    const uint32_t sob = ((S.x < 0.0f ? 1u : 0u) | (S.y < 0.0f ? 2u : 0u) | (S.z < 0.0f ? 4u : 0u)) * c.ostride;
    const uint32_t t0 = path_texel(c, ax + (S.x > 0.0f ? 1 : -1), ay + (S.y > 0.0f ? 1 : -1),
                                   az + (S.z > 0.0f ? 1 : -1), sob);
    f3 ed;
    if (!cert_start(hh.point, ray.dir, S, c.sun_rcp, h.axis, h.eu, ax, ay, az, ed)) {
      CERT_DIAG(6);
      return false;
    }
    const uint32_t n = uint32_t(c.n);
    if (uint32_t(ax) >= n || uint32_t(ay) >= n || uint32_t(az) >= n) { CERT_DIAG(7); return false; }
    if (cert_event<true>(cell_texel(c, ax, ay, az, sob) & kVoxMask, 0u)) { CERT_DIAG(7); return false; }
    const CertResult s = cert_walk<true>(c, hh.point, S, c.sun_rcp, c.max_len - hh.len, ax, ay, az,
                                         h.eu, ed, hh.len, 0u, t0);
    if (s.res == CERT_UNSURE) { CERT_DIAG(8); return false; }
    CERT_DIAG(9);
    brightness = s.res == CERT_HIT ? kAmbient : lit;
  } else {
    CERT_DIAG(4);
  }
  if (!TEX) col = get_color<false>(c, hh);  // textured: the certified texel (cert_texel)
  color.x = mixf(color.x, col.x * col.w * brightness, ray.energy);
  color.y = mixf(color.y, col.y * col.w * brightness, ray.energy);
  color.z = mixf(color.z, col.z * col.w * brightness, ray.energy);
  return true;
}

// RayMarch (voxel.glsl:302-384) of a secondary ray by certified walks; `ray` is inout as in
// march(): leaving a glass medium refracts it in place (:357-380), and the walk restarts from
// that crossing. (cx, cy, cz), e0, ed: the start (cert_start). Returns the first non-air event
// (CERT_HIT), CERT_MISS or CERT_UNSURE.
__device__ __forceinline__ CertResult cert_march(const Ctx& c, Ray& ray, int cx, int cy, int cz, float e0, f3 ed) {
  CertResult h;
  h.res = CERT_UNSURE;
  uint32_t medium = ray.voxel;
  int internal = 0;
  for (int seg = 0; seg < 32; ++seg) {
    if (!fast_path_ok(ray.dir) || !(e0 < kCertMaxOrigin)) { CERT_DIAG(24); return h; }
    const f3 rcp = mk(__builtin_amdgcn_rcpf(ray.dir.x), __builtin_amdgcn_rcpf(ray.dir.y),
                      __builtin_amdgcn_rcpf(ray.dir.z));
    h = cert_walk<false>(c, ray.pos, ray.dir, rcp, c.max_len - ray.len, cx, cy, cz, e0, ed, ray.len,
                         medium);
    if (h.res == CERT_UNSURE) CERT_DIAG(25);
    if (h.res != CERT_HIT || h.byte != 0u) return h;
    CERT_DIAG(30);
    // in-volume refraction at the crossing into the air cell (h.cx, h.cy, h.cz)
    h.res = CERT_UNSURE;
    if (VRT_TREE_CUT & 4) return h;
    const Hit eh = cert_hit_record(ray, h);
    const f3 D0 = ray.dir;
    // the probes at point +- normal/2 (:219-220) read the exact point's cells if the point is
    // robust on the other axes
    const f3 fr = mk(eh.point.x - __builtin_floorf(eh.point.x), eh.point.y - __builtin_floorf(eh.point.y),
                     eh.point.z - __builtin_floorf(eh.point.z));
    const f3 dm = mk(h.eu * __builtin_fabsf(D0.x) + 2e-5f, h.eu * __builtin_fabsf(D0.y) + 2e-5f,
                     h.eu * __builtin_fabsf(D0.z) + 2e-5f);
    if ((h.axis != 0 && !(fr.x >= dm.x && 1.0f - fr.x >= dm.x)) ||
        (h.axis != 1 && !(fr.y >= dm.y && 1.0f - fr.y >= dm.y)) ||
        (h.axis != 2 && !(fr.z >= dm.z && 1.0f - fr.z >= dm.z))) {
      CERT_DIAG(26);
      return h;
    }
    // position-independent directions only (RandomizeDirection's zero-noise identity)
    const float eta = mat_refr(get_voxel(c, eh.point + eh.normal * 0.5f)) /
                      mat_refr(get_voxel(c, eh.point - eh.normal * 0.5f));
    const f3 rd = refract3(normalize3(D0), eh.normal, eta);
    const bool tir = rd.x == 0.0f && rd.y == 0.0f && rd.z == 0.0f;
    if (tir ? !(c.refl_noise == 0.0f && zero_noise_exact(reflect3(D0, eh.normal)))
            : !(c.refr_noise == 0.0f && zero_noise_exact(rd))) {
      CERT_DIAG(27);
      return h;
    }
    Counters kk;
#pragma unroll
    for (int q = 0; q < VRT_CNT_COUNT; ++q) kk.c[q] = 0;
    Ray nr = refraction_ray<false>(c, ray, eh, kk);
    nr.tdepth--;
    if (nr.voxel == medium) {
      internal++;
      if (internal > 10) {
        nr.dir = D0;
        nr.voxel = 0u;
      }
    }
    medium = nr.voxel;
    // restart cell: the crossed cell, or the one before it when the direction turned back
    int nx = h.cx, ny = h.cy, nz = h.cz;
    if ((comp(nr.dir, h.axis) > 0.0f) != (comp(D0, h.axis) > 0.0f)) cell_before(h, D0, nx, ny, nz);
    if (!fast_path_ok(nr.dir)) { CERT_DIAG(28); return h; }
    const f3 rcpn = mk(__builtin_amdgcn_rcpf(nr.dir.x), __builtin_amdgcn_rcpf(nr.dir.y),
                       __builtin_amdgcn_rcpf(nr.dir.z));
    f3 edn;
    if (!cert_start(eh.point, D0, nr.dir, rcpn, h.axis, h.eu, nx, ny, nz, edn)) { CERT_DIAG(28); return h; }
    ray = nr;
    const uint32_t n = uint32_t(c.n);
    if (uint32_t(nx) >= n || uint32_t(ny) >= n || uint32_t(nz) >= n) {
      // out of the volume across the crossed face, moving away: TestCube ends the walk
      h.res = CERT_MISS;
      return h;
    }
    cx = nx;
    cy = ny;
    cz = nz;
    e0 = h.eu;
    ed = edn;
  }
  CERT_DIAG(29);
  h.res = CERT_UNSURE;
  return h;
}

// ------------------------------------------------------------ certified bounce trees --------
//
// The colour of a glass pixel's bounce tree (voxel.glsl:425-452) depends on the exact hit points
// only through the walks' outcomes: reflection and refraction directions, Fresnel energies, the
// sky colour and the brightness are functions of directions and face normals alone
// (:162-165, :203-246, :386-423) once RandomizeDirection is the identity (noise 0, no -0
// component), and the accumulated rayLength enters only through the `< u_MaxRayLength` test. So
// every ray of the tree is walked by a certified walk from its uncertain origin: the parent's
// certified hit, known to its bound eu along the parent (cert_start checks the start cell and
// turns the origin uncertainty into per-axis crossing-order bounds; cert_march carries in-volume
// refraction). Any unsure step sends the whole pixel to the exact path.
//
// A ray in flight is a TreeRay: the Ray the reference would carry (pos and len approximate, dir,
// energy, medium and depths exact) plus its certified start. The DFS keeps the ray the reference
// pops next in registers (the last-pushed child), so only a reflection ray pushed under a
// refraction ray waits, in one per-lane LDS slot; a tree that would hold two such rays at once (never at the BASELINE configs: one glass voxel or
// one-voxel glass walls) goes to the exact path.
struct TreeRay {
  Ray ray;
  int cx, cy, cz;  // start cell (the exact walk's first cell)
  float e0;        // origin uncertainty (parameter along the parent)
  f3 ed;           // per-axis crossing-order uncertainty from it
};
// The slot: 12 words in the lane's own 3 float4s (lane-major; in the in-lane instances the exact
// walk's axis table, c.ax) and 2 words component-major at b[0], b[NL] (there the bounce stack's
// bottom entry): both regions belong to this lane alone, and it is done with the tree before its
// exact path (if any) uses them. (A slot striped over the whole workgroup's pool would overwrite
// the other wave's axis table in the middle of its exact walks.)
constexpr int kTreeWords = 14;
template <int NL>
__device__ __forceinline__ void tree_put(float4* __restrict__ a, float* __restrict__ b, const TreeRay& t) {
  a[0] = make_float4(t.ray.pos.x, t.ray.pos.y, t.ray.pos.z, t.ray.dir.x);
  a[1] = make_float4(t.ray.dir.y, t.ray.dir.z, t.ray.len, t.ray.energy);
  a[2] = make_float4(t.e0, t.ed.x, t.ed.y, t.ed.z);
  // cells in [0, 1024); a stored ray is a reflection ray: medium air
  b[0] = __uint_as_float(uint32_t(t.cx) | uint32_t(t.cy) << 10 | uint32_t(t.cz) << 20);
  b[NL] = __uint_as_float(uint32_t(t.ray.rdepth) | uint32_t(t.ray.tdepth) << 16);
}
template <int NL>
__device__ __forceinline__ TreeRay tree_get(const float4* __restrict__ a, const float* __restrict__ b) {
  TreeRay t;
  const float4 a0 = a[0], a1 = a[1], a2 = a[2];
  t.ray.pos = mk(a0.x, a0.y, a0.z);
  t.ray.dir = mk(a0.w, a1.x, a1.y);
  t.ray.len = a1.z;
  t.ray.energy = a1.w;
  t.e0 = a2.x;
  t.ed = mk(a2.y, a2.z, a2.w);
  const uint32_t w = __float_as_uint(b[0]);
  t.cx = int(w & 1023u);
  t.cy = int((w >> 10) & 1023u);
  t.cz = int((w >> 20) & 1023u);
  const uint32_t dp = __float_as_uint(b[NL]);
  t.ray.rdepth = int(dp & 0xffffu);
  t.ray.tdepth = int(dp >> 16);
  t.ray.voxel = 0u;
  return t;
}

// The certified start of a child ray from the certified hit h of its parent (direction d0 there):
// the start cell, checked inside the volume, and cert_start's bounds. false: unsure.
__device__ __forceinline__ bool tree_start(const Ctx& c, const CertResult& h, const Hit& hh, const f3 d0,
                                           TreeRay& t) {
  if (!fast_path_ok(t.ray.dir)) return false;
  const uint32_t n = uint32_t(c.n);
  if (uint32_t(t.cx) >= n || uint32_t(t.cy) >= n || uint32_t(t.cz) >= n) { CERT_DIAG(31); return false; }
  const f3 rn = mk(__builtin_amdgcn_rcpf(t.ray.dir.x), __builtin_amdgcn_rcpf(t.ray.dir.y),
                   __builtin_amdgcn_rcpf(t.ray.dir.z));
  t.e0 = h.eu;
  return cert_start(hh.point, d0, t.ray.dir, rn, h.axis, h.eu, t.cx, t.cy, t.cz, t.ed);
}

// GetReflectionRay (voxel.glsl:203-215) of a certified hit: the direction must not depend on the
// point (RandomizeDirection's zero-noise identity); it starts back in the cell before the face
template <bool TEX>
__device__ __forceinline__ bool tree_reflection(const Ctx& c, const Ray& ray, const CertResult& h, const Hit& hh,
                                                TreeRay& t) {
  if (!(c.refl_noise == 0.0f && zero_noise_exact(reflect3(ray.dir, hh.normal)))) return false;
  if (VRT_TREE_CUT & 1) return false;
  t.ray = reflection_ray(c, ray, hh);
  cell_before(h, ray.dir, t.cx, t.cy, t.cz);
  return tree_start(c, h, hh, ray.dir, t);
}

// GetRefractionRay (voxel.glsl:217-246) of a certified hit: the probes at point +- normal / 2
// (:219-220) read the exact point's cells when the point is robust on the other axes (cert_start
// checks it); total internal reflection turns it into the reflection ray, back before the face
template <bool TEX>
__device__ __forceinline__ bool tree_refraction(const Ctx& c, const Ray& ray, const CertResult& h, const Hit& hh,
                                                TreeRay& t) {
  if (VRT_TREE_CUT & 2) return false;
  const float eta = mat_refr(get_voxel(c, hh.point + hh.normal * 0.5f)) /
                    mat_refr(get_voxel(c, hh.point - hh.normal * 0.5f));
  const f3 rd = refract3(normalize3(ray.dir), hh.normal, eta);
  const bool tir = rd.x == 0.0f && rd.y == 0.0f && rd.z == 0.0f;
  if (tir ? !(c.refl_noise == 0.0f && zero_noise_exact(reflect3(ray.dir, hh.normal)))
          : !(c.refr_noise == 0.0f && zero_noise_exact(rd)))
    return false;
  Counters kk;
#pragma unroll
  for (int q = 0; q < VRT_CNT_COUNT; ++q) kk.c[q] = 0;
  t.ray = refraction_ray<TEX>(c, ray, hh, kk);
  t.cx = h.cx;  // into the hit cell, or (total internal reflection) back before it
  t.cy = h.cy;
  t.cz = h.cz;
  if ((comp(t.ray.dir, h.axis) > 0.0f) != (comp(ray.dir, h.axis) > 0.0f)) cell_before(h, ray.dir, t.cx, t.cy, t.cz);
  return tree_start(c, h, hh, ray.dir, t);
}

// One ray of a certified tree: the colour update of `ray`'s walk outcome h, its children, then the
// walk of the ray the reference pops next (ray, h updated). kTreeDone: the tree is complete (colour
// final); kTreeUnsure: it cannot be certified (colour meaningless); kTreeNext: continue with ray, h.
constexpr int kTreeNext = 0, kTreeDone = 1, kTreeUnsure = -1;
template <int NL>
__device__ __forceinline__ int tree_step(const Ctx& c, int max_refl, int max_transp, Ray& ray, CertResult& h,
                                         f3& color, bool& pending, float4* __restrict__ lta,
                                         float* __restrict__ ltb) {
  // the sun vector opaque per ray, as in the exact path's bounce loop (trace_with_shadow): else
  // the shadow walk's per-sun products are hoisted into VGPRs live across the whole tree and
  // spilled on its entry
  Ctx lc = c;
  asm volatile("" : "+s"(lc.sun_n.x), "+s"(lc.sun_n.y), "+s"(lc.sun_n.z), "+s"(lc.sun_rcp.x),
               "+s"(lc.sun_rcp.y), "+s"(lc.sun_rcp.z));
  bool next = false;
  TreeRay t;
  CTRACE(c, 200, h.res, h.byte, h.axis, h.u, h.eu, ray.rdepth, ray.tdepth);
  CTRACE(c, 201, ray.pos.x, ray.pos.y, ray.pos.z, ray.dir.x, ray.dir.y, ray.dir.z, ray.len);
  CTRACE(c, 202, color.x, color.y, color.z, ray.energy, h.cx, h.cy, h.cz);
  if (h.res == CERT_MISS) {
    apply_sky_color(c, ray, color);
  } else {
    const Hit hh = cert_hit_record(ray, h);
    if (!cert_shade_hit<false>(lc, ray, h, hh, color)) { CERT_DIAG(22); return kTreeUnsure; }
    // children (:440-448): the reflection ray is pushed first, the refraction ray second and
    // popped first; the stack (R + T + 1 entries) never fills with at most one ray waiting
    const uint32_t m = mat_id(h.byte);
    const bool pr = mat_reflective(m) && ray.rdepth < max_refl;
    const bool pt = mat_transparent(m) && ray.tdepth < max_transp && get_color<false>(c, hh).w != 1.0f;
    if (pr && pt) {
      if (pending) { CERT_DIAG(18); return kTreeUnsure; }
      TreeRay r;
      if (!tree_reflection<false>(c, ray, h, hh, r)) { CERT_DIAG(19); return kTreeUnsure; }
      tree_put<NL>(lta, ltb, r);
      pending = true;
      if (!tree_refraction<false>(c, ray, h, hh, t)) { CERT_DIAG(20); return kTreeUnsure; }
      next = true;
    } else if (pr) {
      if (!tree_reflection<false>(c, ray, h, hh, t)) { CERT_DIAG(19); return kTreeUnsure; }
      next = true;
    } else if (pt) {
      if (!tree_refraction<false>(c, ray, h, hh, t)) { CERT_DIAG(20); return kTreeUnsure; }
      next = true;
    }
  }
  if (!next) {
    if (!pending) { CERT_DIAG(17); return kTreeDone; }
    pending = false;
    t = tree_get<NL>(lta, ltb);
  }
  ray = t.ray;
  h = cert_march(c, ray, t.cx, t.cy, t.cz, t.e0, t.ed);
  if (h.res == CERT_UNSURE) { CERT_DIAG(21); return kTreeUnsure; }
  CERT_DIAG(23);
  return kTreeNext;
}

// The bounce tree of a glass primary hit h0 of ray0 (fragment main, voxel.glsl:425-452) by
// certified walks, colour folded in the reference's DFS order as TraceWithShadow does (:395-423):
// each ray's RayMarch by cert_march, its hit shaded with a certified shadow (none for glass), a
// miss with the sky colour. Colour-only (TEX false) frames. Returns false, colour untouched, when
// any walk, start or direction could differ from the exact path's.
// (Walking the primary ray through this loop too, one walk call site for every ray, made the
// certified pass 3x slower: every pixel then carried the tree's registers; r06_s4.)
// lta / ltb: this lane's LDS slot (tree_put; NL lanes per workgroup).
template <int NL>
__device__ __forceinline__ bool cert_tree(const Ctx& c, int max_refl, int max_transp, const Ray& ray0,
                                          const CertResult& h0, f3& color_out, float4* __restrict__ lta,
                                          float* __restrict__ ltb) {
  f3 color = mk(0.0f, 0.0f, 0.0f);
  Ray ray = ray0;
  CertResult h = h0;
  bool pending = false;  // a reflection ray waits in the LDS slot
  CERT_DIAG(16);
  for (;;) {
    const int r = tree_step<NL>(c, max_refl, max_transp, ray, h, color, pending, lta, ltb);
    if (r == kTreeUnsure) return false;
    if (r == kTreeDone) break;
  }
  color_out = color;
  return true;
}

// The exact walk's start cell from P along D (voxel.glsl:306-309: first planes d < 0 ? ceil(p - 1)
// : floor(p + 1)); false when it lies outside the volume or a plane disagrees with the cell's.
__device__ __forceinline__ bool exact_start_cell(const Ctx& c, const f3 P, const f3 D, int& cx, int& cy,
                                                 int& cz) {
  const int sx = D.x > 0.0f ? 1 : -1, sy = D.y > 0.0f ? 1 : -1, sz = D.z > 0.0f ? 1 : -1;
  cx = sx > 0 ? int(__builtin_floorf(P.x)) : int(__builtin_ceilf(P.x)) - 1;
  cy = sy > 0 ? int(__builtin_floorf(P.y)) : int(__builtin_ceilf(P.y)) - 1;
  cz = sz > 0 ? int(__builtin_floorf(P.z)) : int(__builtin_ceilf(P.z)) - 1;
  const float wpx = sx > 0 ? __builtin_floorf(P.x + 1.0f) : __builtin_ceilf(P.x - 1.0f);
  const float wpy = sy > 0 ? __builtin_floorf(P.y + 1.0f) : __builtin_ceilf(P.y - 1.0f);
  const float wpz = sz > 0 ? __builtin_floorf(P.z + 1.0f) : __builtin_ceilf(P.z - 1.0f);
  const uint32_t n = uint32_t(c.n);
  if (uint32_t(cx) >= n || uint32_t(cy) >= n || uint32_t(cz) >= n) return false;
  return wpx == float(cx + (sx > 0)) && wpy == float(cy + (sy > 0)) && wpz == float(cz + (sz > 0));
}

// Cells the exact walk samples behind its start cell. A start coordinate P_a that is an integer k
// with D_a < 0 (a shadow or secondary ray from an exact hit point on its face plane) makes the
// start cell k - 1 on axis a, but until cur_a = P_a + s D_a rounds off k the exact walk samples
// layer k — beyond the plane — at every crossing of another axis (r02 s18: a shadow ray from
// (33.000008, 127, 37.02) going -x, -y sampled the panel voxel (32, 127, 37) at its x crossing
// 8.5e-6 after the start; the certified walk had jumped that crossing). The certified walk cannot
// see those cells, so they are checked here: every cell of layer k the walk may enter across an
// axis crossed within 2 ulp(k) / |D_a| (+1e-5) of the start must be a non-event, else unsure.
template <bool SHADOW>
__device__ __forceinline__ bool start_layers_clear(const Ctx& c, const f3 P, const f3 D, int cx, int cy,
                                                   int cz, uint32_t medium) {
  const float p[3] = {P.x, P.y, P.z}, d[3] = {D.x, D.y, D.z};
  const int cell[3] = {cx, cy, cz};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (!(d[a] < 0.0f) || p[a] != __builtin_floorf(p[a])) continue;
    const float off = (0x1p-22f * __builtin_fmaxf(__builtin_fabsf(p[a]), 1.0f) + 1e-5f) / __builtin_fabsf(d[a]);
    // two crossings of one axis b in layer k (a nearly parallel D_a keeps cur_a on k: a
    // straight-down lattice camera's ray at x = 64 with D_x = -2.2e-8 read plane N's GL_REPEAT
    // copy for 170 units) need off >= 1 / |D_b| >= 1: more cells than checked here, unsure
    if (off >= 1.0f) return false;
    int q[3] = {cell[0], cell[1], cell[2]};
    q[a] += 1;  // layer k
    bool early[3] = {false, false, false};
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      if (b == a) continue;
      const float plane = float(cell[b] + (d[b] > 0.0f ? 1 : 0));
      early[b] = (plane - p[b]) / d[b] < off;  // first crossing of axis b
    }
    const int b1 = a == 0 ? 1 : 0, b2 = a == 2 ? 1 : 2;
    const int s1 = d[b1] > 0.0f ? 1 : -1, s2 = d[b2] > 0.0f ? 1 : -1;
    // shadow walks: the exact walk may cross b in layer k and so never sample the start layer's
    // cell across b, which the certified walk reaches by that crossing and, if it blocks,
    // reports as a hit "whichever way the walk goes" (a straight-down lattice camera's shadow
    // from x = 33.0 going -x sampled (33, 30, 2) at its z crossing and never the solid (32, 30,
    // 2)): unsure whenever a crossing falls in the sliver
    if (SHADOW && (early[b1] || early[b2])) return false;
    int r[3];
    if (early[b1]) {
      r[0] = q[0]; r[1] = q[1]; r[2] = q[2]; r[b1] += s1;
      if (cert_event<SHADOW>(alt_byte(c, r[0], r[1], r[2], 0u), medium)) return false;
    }
    if (early[b2]) {
      r[0] = q[0]; r[1] = q[1]; r[2] = q[2]; r[b2] += s2;
      if (cert_event<SHADOW>(alt_byte(c, r[0], r[1], r[2], 0u), medium)) return false;
    }
    if (early[b1] && early[b2]) {
      r[0] = q[0]; r[1] = q[1]; r[2] = q[2]; r[b1] += s1; r[b2] += s2;
      if (cert_event<SHADOW>(alt_byte(c, r[0], r[1], r[2], 0u), medium)) return false;
    }
  }
  return true;
}

// The shadow bit of an exact hit h by a certified walk: the shadow ray starts at the exact hit
// point h.point with len h.len (GetShadowRay, :191-201), so its start is known exactly, as a
// primary ray's is (e0 = 0, the exact walk's own start cell). 1 blocked, 0 lit, -1 unsure.
__device__ __forceinline__ int cert_shadow_exact(const Ctx& c, const Hit& h) {
  const f3 S = c.sun_n;
  int cx, cy, cz;
  if (!fast_path_ok(S) || !exact_start_cell(c, h.point, S, cx, cy, cz)) return -1;
  if (!start_layers_clear<true>(c, h.point, S, cx, cy, cz, 0u)) return -1;
  const CertResult s = cert_walk<true>(c, h.point, S, c.sun_rcp, c.max_len - h.len, cx, cy, cz, 0.0f,
                                       mk(0.0f, 0.0f, 0.0f), h.len, 0u);
  return s.res == CERT_UNSURE ? -1 : (s.res == CERT_HIT ? 1 : 0);
}

// An air segment of a bounce-stack ray by a certified walk from the exact point ray.pos (len
// ray.len) in cell (cx, cy, cz); ed: per-axis crossing-order uncertainty of the exact walk's
// planes. In an air medium every event is a hit (:353), and a non-glass hit spawns no rays
// (:440-448). true (colour updated as TraceWithShadow's, :395-423): a miss, or a non-glass hit
// whose shadow certifies. false (colour untouched): the exact march goes on.
__device__ __forceinline__ bool cert_air_segment(const Ctx& c, const Ray& ray, int cx, int cy, int cz,
                                                 const f3 ed, f3& color) {
  const f3 D = ray.dir;
  const f3 rcp = mk(__builtin_amdgcn_rcpf(D.x), __builtin_amdgcn_rcpf(D.y), __builtin_amdgcn_rcpf(D.z));
  const CertResult h = cert_walk<false>(c, ray.pos, D, rcp, c.max_len - ray.len, cx, cy, cz, 0.0f, ed,
                                        ray.len, 0u);
  if (h.res == CERT_UNSURE) return false;
  if (h.res == CERT_MISS) {
    apply_sky_color(c, ray, color);
    return true;
  }
  if (mat_id(h.byte) == 2u) return false;
  return cert_shade_hit(c, ray, h, cert_hit_record(ray, h), color);
}

// A secondary ray from an exact origin (the reflection or refraction ray of an exact hit) in air:
// its walk certifies as a primary's does
__device__ __forceinline__ bool cert_secondary(const Ctx& c, const Ray& ray, f3& color) {
  int cx, cy, cz;
  if (ray.voxel != 0u || !fast_path_ok(ray.dir) || !exact_start_cell(c, ray.pos, ray.dir, cx, cy, cz) ||
      !start_layers_clear<false>(c, ray.pos, ray.dir, cx, cy, cz, 0u))
    return false;
  return cert_air_segment(c, ray, cx, cy, cz, mk(0.0f, 0.0f, 0.0f), color);
}

// The rest of a march after an in-volume refraction into air at the exact crossing w.cur of axis
// fa (march, :357-380): the exact walk goes on from pos = cur, len0 = w.len, with the first
// planes initial_t's on the other axes and cur_fa + sign on axis fa. That plane lies within
// delta = |(cur_fa + sign) - (k + sign)| of the lattice plane (k = rint(cur_fa)), and every later
// axis-fa plane of the walk (cur_fa + sign at each crossing) keeps that offset: the certified walk
// starts in the cell beyond k and takes delta |1/d_fa| (doubled) as that axis's crossing-order
// uncertainty. The step cap (VRT_MAX_STEPS per march) must be out of reach: <= 3N + 4 more steps.
__device__ __forceinline__ bool cert_continuation(const Ctx& c, const Ray& ray, const WalkState& w, int fa,
                                                  f3& color) {
  const f3 D = ray.dir, P = ray.pos;
  if (!fast_path_ok(D) || w.it + 3u * uint32_t(c.n) + 16u > uint32_t(VRT_MAX_STEPS)) return false;
  int cx, cy, cz;
  const float pa = comp(P, fa), da = comp(D, fa);
  const float k = __builtin_rintf(pa);
  const float sa = da > 0.0f ? 1.0f : -1.0f;
  const float delta = __builtin_fabsf((pa + sa) - (k + sa));
  if (!(delta < 1e-3f)) return false;
  // the other axes as a fresh walk's start; axis fa replaced below
  {
    const int sx = D.x > 0.0f ? 1 : -1, sy = D.y > 0.0f ? 1 : -1, sz = D.z > 0.0f ? 1 : -1;
    cx = sx > 0 ? int(__builtin_floorf(P.x)) : int(__builtin_ceilf(P.x)) - 1;
    cy = sy > 0 ? int(__builtin_floorf(P.y)) : int(__builtin_ceilf(P.y)) - 1;
    cz = sz > 0 ? int(__builtin_floorf(P.z)) : int(__builtin_ceilf(P.z)) - 1;
    const float wpx = sx > 0 ? __builtin_floorf(P.x + 1.0f) : __builtin_ceilf(P.x - 1.0f);
    const float wpy = sy > 0 ? __builtin_floorf(P.y + 1.0f) : __builtin_ceilf(P.y - 1.0f);
    const float wpz = sz > 0 ? __builtin_floorf(P.z + 1.0f) : __builtin_ceilf(P.z - 1.0f);
    if ((fa != 0 && wpx != float(cx + (sx > 0))) || (fa != 1 && wpy != float(cy + (sy > 0))) ||
        (fa != 2 && wpz != float(cz + (sz > 0))))
      return false;
    const int ka = int(k) - (da > 0.0f ? 0 : 1);
    if (fa == 0) cx = ka;
    else if (fa == 1) cy = ka;
    else cz = ka;
  }
  const uint32_t n = uint32_t(c.n);
  if (uint32_t(cx) >= n || uint32_t(cy) >= n || uint32_t(cz) >= n) return false;
  // the start cell lies beyond plane k on axis fa, but P_fa may lie before it (by up to delta) or
  // on it: until cur_fa = P_fa + s D_fa is past k, the exact walk samples the layer before k at
  // every crossing of another axis (as start_layers_clear's layer k for a start on a plane), which
  // the certified walk does not see (a glass cube's face voxel beside the refraction point,
  // sampled 3.7e-6 after the start, made a lattice camera's pixel differ before this test):
  // unsure when another axis is crossed that early. By the hardware reciprocal (<= 1 ulp) against
  // a bound widened past its error: never fewer cases than the exact quotients would give.
  {
    const float before = __builtin_fmaxf((k - pa) * sa, 0.0f);
    const float off = (before + 0x1p-22f * __builtin_fmaxf(__builtin_fabsf(pa), 1.0f) + 1e-5f) *
                      __builtin_fabsf(__builtin_amdgcn_rcpf(da)) * 1.00002f;
    const float tx = fa == 0 ? off : (float(cx + (D.x > 0.0f ? 1 : 0)) - P.x) * __builtin_amdgcn_rcpf(D.x);
    const float ty = fa == 1 ? off : (float(cy + (D.y > 0.0f ? 1 : 0)) - P.y) * __builtin_amdgcn_rcpf(D.y);
    const float tz = fa == 2 ? off : (float(cz + (D.z > 0.0f ? 1 : 0)) - P.z) * __builtin_amdgcn_rcpf(D.z);
    if (__builtin_fminf(tx, __builtin_fminf(ty, tz)) < off) return false;
  }
  f3 ed = mk(0.0f, 0.0f, 0.0f);
  set_comp(ed, fa, 2.0f * delta * __builtin_fabsf(__builtin_amdgcn_rcpf(da)) + 1e-6f);
  return cert_air_segment(c, ray, cx, cy, cz, ed, color);
}

// RayMarch + TraceWithShadow of a bounce-stack ray (stats-free, colour-only) with its air
// segments — the whole ray from its exact origin, or the rest after an in-volume refraction into
// air — settled by certified walks where they can be (settled: colour updated, no secondary
// rays); the exact march (as march()) otherwise.
// (Out of line it costs C2-C4 +45 %, profiles/r01_v69_ab_noinline_w6.log.)
__device__ __forceinline__ Hit march_cert(const Ctx& c, Ray& ray, f3& color, bool& settled, Counters& k,
                          uint32_t& steps, uint32_t& flags) {
  Hit h;
  h.found = false;
  h.vidx = -1;
  h.len = 0.0f;
  h.voxel = 0;
  h.point = mk(0.0f, 0.0f, 0.0f);
  h.normal = h.point;
  h.axis = 0;
  settled = cert_secondary(c, ray, color);
  if (settled) return h;
  WalkState w;
  walk_init(w, ray);
  uint32_t medium = ray.voxel;
  int internal = 0;
  for (;;) {
    int axis;
    int32_t vidx;
    uint32_t v;
    const int r = walk_ray<false>(c, ray.pos, ray.dir, ray.len, medium, w, axis, vidx, v);
    if (r != WALK_EVENT) break;
    f3 normal = mk(0.0f, 0.0f, 0.0f);
    set_comp(normal, axis, -gsign(comp(ray.dir, axis)));
    if (v != 0u) {
      h.found = true;
      h.voxel = v;
      h.vidx = vidx;
      h.point = w.cur;
      h.len = w.len;
      h.normal = normal;
      h.axis = axis;
      break;
    }
    Hit e;
    e.found = true;
    e.voxel = 0;
    e.vidx = vidx;
    e.point = w.cur;
    e.len = w.len;
    e.normal = normal;
    e.axis = axis;
    const f3 old_dir = ray.dir;
    ray = refraction_ray<false>(c, ray, e, k);
    ray.tdepth--;
    if (ray.voxel == medium) {
      internal++;
      if (internal > 10) {
        ray.dir = old_dir;
        ray.voxel = 0;
      }
    }
    medium = ray.voxel;
    w.t = initial_t(ray.dir, w.cur, ray.pos);
    const f3 step = sign3(ray.dir);
    const float q = ((comp(w.cur, axis) + comp(step, axis)) - comp(ray.pos, axis)) /
                        comp(ray.dir, axis) - (w.len - ray.len);
    set_comp(w.t, axis, q);
    if (medium == 0u && cert_continuation(c, ray, w, axis, color)) {
      settled = true;
      return h;
    }
  }
  return h;
}

// The whole pixel by certified walks, when it can be certified: a primary miss, or a non-glass
// primary hit with its shadow. The pixel's colour starts black (voxel.glsl:428); color_out is
// written only when the pixel certifies. false when any walk or any derived value could differ
// from the exact path's, or the hit is glass (its secondary rays start at the exact hit point):
// the pixel then takes the exact path.
// Textured mode: the texel GetColor (voxel.glsl:174-182) reads at the exact hit point, from the
// certified hit. The exact hit point is currentPos of the exact walk's hit step; on each face axis
// it lies within delta = eu |D_b| + the roundings of both points' pos + s dir of the certified
// point (eu bounds the exact walk's parameter there, cert_gamma). get_color's texel index is a
// composition of correctly rounded monotone operations of the coordinate (frac by floor, + texX,
// x ts, / S, floor(. x S)), so if both ends of [p - delta, p + delta] lie in the same voxel and give
// the same texel, every point between does: the exact texel is that one. false: unsure.
__device__ __forceinline__ bool texel_pair(const Ctx& c, float p, float d, uint32_t slot, bool flip, uint32_t& t) {
  const float lo = p - d, hi = p + d;
  if (__builtin_floorf(lo) != __builtin_floorf(hi)) return false;
  auto idx = [&](float q) {
    const float f = q - floorf(q);
    if (!flip) {  // tx = ((fx + texX) * ts) / S, u = tx
      const float u = ((f + float(slot)) * c.atlas_fts) / c.atlas_fs;
      return cvt_flr(u * c.atlas_fs) & c.atlas_mask;
    }
    const float ty = (((1.0f - f) + float(slot)) * c.atlas_fts) / c.atlas_fs;  // v = 1 - ty
    return cvt_flr((1.0f - ty) * c.atlas_fs) & c.atlas_mask;
  };
  t = idx(lo);
  return t == idx(hi);
}

__device__ __forceinline__ bool cert_texel(const Ctx& c, const Ray& ray, const CertResult& h, const Hit& hh,
                                           float4& col) {
  const uint32_t m = mat_id(h.byte);
  const float px = hh.axis == 0 ? hh.point.z : hh.point.x;  // intersectionAxis[a][1]
  const float py = hh.axis == 2 ? hh.point.y : (hh.axis == 1 ? hh.point.z : hh.point.y);  // [a][2]
  const float dx = hh.axis == 0 ? ray.dir.z : ray.dir.x;
  const float dy = hh.axis == 2 ? ray.dir.y : (hh.axis == 1 ? ray.dir.z : ray.dir.y);
  const float px0 = hh.axis == 0 ? ray.pos.z : ray.pos.x;
  const float py0 = hh.axis == 2 ? ray.pos.y : (hh.axis == 1 ? ray.pos.z : ray.pos.y);
  // eu along the ray, plus 2 ulp-scale roundings of each point's P + s D (both points), doubled
  const float ex = h.eu * __builtin_fabsf(dx) +
                   0x1p-21f * (__builtin_fabsf(px0) + __builtin_fabsf(h.u * dx) + __builtin_fabsf(px) + 1.0f);
  const float ey = h.eu * __builtin_fabsf(dy) +
                   0x1p-21f * (__builtin_fabsf(py0) + __builtin_fabsf(h.u * dy) + __builtin_fabsf(py) + 1.0f);
  uint32_t i, j;
  if (!texel_pair(c, px, ex, mat_tex_x(m), false, i) || !texel_pair(c, py, ey, mat_tex_y(m), true, j)) return false;
  const uint32_t t = c.atlas[j * (c.atlas_mask + 1u) + i];
  col = make_float4(float(t & 0xFFu) / 255.0f, float((t >> 8) & 0xFFu) / 255.0f,
                    float((t >> 16) & 0xFFu) / 255.0f, float(t >> 24) / 255.0f);
  return true;
}

// TREE (colour-only): a glass primary hit's bounce tree by certified walks too (cert_tree; ltb and c.ax its
// LDS slot), instead of leaving the whole pixel to the exact path.
// us_out: the primary walk's certified prefix (CertResult::us) for the exact path, -1 if none.
template <bool TEX = false, bool TREE = false, int NL = kWgThreads>
__device__ __forceinline__ bool cert_pixel(const Ctx& c, const Ray& ray0, f3& color_out, int max_refl = 0,
                                           int max_transp = 0, float* __restrict__ ltb = nullptr,
                                           float* us_out = nullptr) {
  const f3 P = ray0.pos, D = ray0.dir;
  if (VRT_DIAG_PHASE <= 1) {
    color_out = D;
    return true;
  }
  if (!fast_path_ok(D)) { CERT_DIAG(0); return false; }
  int cx, cy, cz;
  if (!exact_start_cell(c, P, D, cx, cy, cz) || !start_layers_clear<false>(c, P, D, cx, cy, cz, 0u)) {
    CERT_DIAG(0);
    return false;
  }
  // hardware reciprocals (<= 1 ulp): the certified walk only needs its own error bounded
  const f3 rcp = mk(__builtin_amdgcn_rcpf(D.x), __builtin_amdgcn_rcpf(D.y), __builtin_amdgcn_rcpf(D.z));
  CertResult h = cert_walk<false>(c, P, D, rcp, c.max_len - ray0.len, cx, cy, cz, 0.0f,
                                  mk(0.0f, 0.0f, 0.0f), 0.0f, 0u);
  if (us_out) *us_out = h.us;
#ifdef VRT_CERT_DIAG
  cert_diag_iters(10, h.iters);
#endif
  if (VRT_DIAG_PHASE == 2) {
    color_out = mk(float(h.res), float(h.byte), h.u);
    return true;
  }
  if (h.res == CERT_UNSURE) { CERT_DIAG(1); return false; }
  f3 color = mk(0.0f, 0.0f, 0.0f);
  if (h.res == CERT_MISS) {
    CERT_DIAG(2);
    apply_sky_color(c, ray0, color);
    color_out = color;
    return true;
  }
  if (mat_id(h.byte) == 2u) {  // only glass spawns secondary rays (:440-448)
    CERT_DIAG(3);
    if constexpr (TREE && !TEX) return cert_tree<NL>(c, max_refl, max_transp, ray0, h, color_out, c.ax, ltb);
    return false;
  }
  const Hit hh = cert_hit_record(ray0, h);
  float4 col = float4();
  if (TEX && !cert_texel(c, ray0, h, hh, col)) return false;
  if (!cert_shade_hit<TEX>(c, ray0, h, hh, color, col)) return false;
  color_out = color;
  return true;
}

// ---- RGB8 framebuffer store + temporal filter (oracle/vrt_oracle.c oracle_temporal) ----------
// GL float -> UNORM8 store into the RGB8 FBO attachments (FrameBuffer.cpp:8): clamp to [0,1]
// (NaN -> 0), scale by 255, round half to even (pinned in DESIGN.md); a texel reads back b / 255.
__device__ __forceinline__ uint32_t unorm8(float f) {
  const float c = __builtin_fminf(__builtin_fmaxf(f, 0.0f), 1.0f);
  return uint32_t(__builtin_rintf(c * 255.0f));
}
// b / 255 rounded correctly, as q0 = b * RN(1/255) plus one fma correction: equal to the IEEE
// division for every byte (exhaustive check, tests/test_div255.py)
__device__ __forceinline__ float unorm8_read(uint32_t b) {
  const float a = float(b), y = 1.0f / 255.0f;
  const float q0 = a * y;
  return __builtin_fmaf(__builtin_fmaf(-255.0f, q0, a), y, q0);
}
__device__ __forceinline__ uint32_t pack_rgb8(float r, float g, float b) {
  return unorm8(r) | (unorm8(g) << 8) | (unorm8(b) << 16) | 0xFF000000u;
}
// temporal.glsl:18  color = u_Alpha * newColor + (1 - u_Alpha) * averageColor, on RGB8 texels
__device__ __forceinline__ uint32_t temporal_blend(uint32_t nw, uint32_t old, float alpha) {
  const float om = 1.0f - alpha;
  uint32_t r = 0xFF000000u;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float v = alpha * unorm8_read((nw >> (8 * ch)) & 0xFFu) + om * unorm8_read((old >> (8 * ch)) & 0xFFu);
    r |= unorm8(v) << (8 * ch);
  }
  return r;
}

// Lane id as a fresh (volatile) value each call, so the compiler cannot keep one copy alive
// across the whole trace.
__device__ __forceinline__ uint32_t lane_id() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
// kWgWaves waves per workgroup (vrt_internal.h), each rendering an 8x8 pixel tile: a workgroup
// covers kTileW x kTileH pixels (wave = threadIdx.x >> 6, uniform). Tiles are dispatched in row
// order (an XCD-aware order that
// keeps runs of tiles on one XCD's L2 was neutral or worse, profiles/r01_v29_ab_xcd_tile_swizzle_negative.log).

// Heavy tiles first (vrt_set_tile_order). A frame ends with its longest waves, those with exact-path
// pixels (glass bounce stacks, walks the certified walk could not settle); dispatched in row
// order, they start wherever they are in the image. Each stats-free launch therefore records which
// of its tiles had such a pixel (until r02: only bounce stacks; C3 -2 %, profiles/r02_s09), and the
// next launch of the same band (same stream) dispatches those first.
// Workgroups are dealt to the 8 XCDs round-robin (workgroup L on XCD L % 8), and a tile keeps its
// XCD — its L2 — from launch to launch only if it keeps its slot's residue mod 8: every
// permutation that ignored this was 9-60 % slower at C3 (profiles/r02_s12_tileperm, r02_s14).
// So heavy tiles are listed per class r = tile % 8: as a heavy tile finishes, its last wave
// appends it to its class's list (kOrdClasses counters, one 256-byte line each) and stores its
// rank (list position + 1; 0 for the other tiles). The next launch's grid is 8*ord_q + tiles
// workgroups: slot L < 8*ord_q renders entry n - 1 - L / 8 of class L % 8's list (n = its length,
// at most ord_q) if L / 8 < n, else exits — the class's heavy tiles in reverse completion order,
// those that finished last first (C3 -4 % against completion order and against the flag passes,
// profiles/r02_s14); slot 8*ord_q + t renders tile t unless its rank is in [1, ord_q] (rendered by
// the first pass). The list and the ranks of a launch are written together, so every tile is rendered
// exactly once (a fresh zeroed buffer: no heavy tiles). Until r02 s14 the first pass was `tiles`
// workgroups testing per-tile flags (same slot residues), most of them empty.
__device__ __forceinline__ uint32_t* ord_ctr(const KArgs& a, uint32_t set, uint32_t r) {
  return a.order + (set * kOrdClasses + r) * kOrdCtrStride;
}
__device__ __forceinline__ uint32_t* ord_rank(const KArgs& a, uint32_t set) {
  return a.order + kOrdHdr + (1u + set) * a.tiles;
}
__device__ __forceinline__ uint32_t* ord_list(const KArgs& a, uint32_t set) {  // entry j of class r: [j*8 + r]
  return a.order + kOrdHdr + 3u * a.tiles + set * (a.tiles + kOrdClasses);
}
// The tile workgroup L renders, or ~0u (nothing to do)
__device__ __forceinline__ uint32_t ordered_tile(const KArgs& a, uint32_t L) {
  const uint32_t cap = kOrdClasses * a.ord_q;
  if (L < cap) {
    const uint32_t r = L % kOrdClasses, j = L / kOrdClasses;
    if (j == 0u && threadIdx.x == 0u) *ord_ctr(a, a.ctr_z, r) = 0u;  // for the launch after the next
    const uint32_t n = min(*ord_ctr(a, a.ctr_r, r), a.ord_q);
    return j < n ? ord_list(a, a.ord_r)[(n - 1u - j) * kOrdClasses + r] : ~0u;  // last finished first
  }
  const uint32_t t = L - cap;
  return ord_rank(a, a.ord_r)[t] - 1u < a.ord_q ? ~0u : t;  // rank 0 wraps to ~0u: not listed
}
// after the trace: the tile's last wave files it for the next launch
// (counter: bits 0-7 waves done, 8-15 heavy waves)
__device__ __forceinline__ void order_record(const KArgs& a, uint32_t tile, bool heavy_wave) {
  uint32_t* cnt = a.order + kOrdHdr + tile;
  const uint32_t add = 1u | (heavy_wave ? 0x100u : 0u);
  const uint32_t old = atomicAdd(cnt, add);
  if ((old & 0xFFu) != uint32_t(kWgWaves) - 1u) return;
  *cnt = 0u;
  uint32_t rank = 0u;
  if (((old + add) & 0xFF00u) != 0u) {
    const uint32_t r = tile % kOrdClasses;
    const uint32_t k = atomicAdd(ord_ctr(a, a.ctr_w, r), 1u);  // <= tiles / 8: one per tile of class r
    ord_list(a, a.ord_w)[k * kOrdClasses + r] = tile;
    rank = k + 1u;
  }
  ord_rank(a, a.ord_w)[tile] = rank;
}

__device__ __forceinline__ int pixel_x(uint32_t tx, int wave, uint32_t lane) {
  return int(tx) * kTileW + (wave & 1) * 8 + int(lane & 7u);
}
__device__ __forceinline__ int pixel_row(uint32_t ty, int wave, uint32_t lane) {
  return int(ty) * kTileH + (wave >> 1) * 8 + int(lane >> 3);
}
// frame row of band row li: blocks of 2^row_blk_sh adjacent rows, row_step rows apart (ABI v11);
// row_blk_sh = 0 is the cyclic-row band row0 + li * row_step
__device__ __forceinline__ int frame_row(const KArgs& a, int li) {
  return a.row0 + (li >> a.row_blk_sh) * a.row_step + (li & ((1 << a.row_blk_sh) - 1));
}

#ifdef VRT_STAMPS
// Diagnostic build only (scripts/stamps.py): per wave {start, end} s_memrealtime (100 MHz) and
// {HW_ID, XCC_ID}, indexed by the linear wave id. Never part of the product library.
constexpr int kMaxStampWaves = 1 << 18;
__device__ unsigned long long g_stamps[kMaxStampWaves][3];
// {time after the certified attempt (all lanes reconverged), lanes that took the exact path}
__device__ unsigned long long g_stamps2[kMaxStampWaves][2];
// exact_pass_kernel, per workgroup: {start, end, XCC_ID << 32 | HW_ID, pixels | dense << 16}
__device__ unsigned long long g_stamps4[kMaxStampWaves][4];

__device__ __forceinline__ uint32_t hw_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  return v;
}
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v;
}
#endif

// Counters (STATS launches): one 64-bit add per wave and counter into replica
// (block % kCntReplicas); a single array would serialise ~300K same-address atomics per 1080p
// frame at the memory side.

// Waves per SIMD the register budget is sized for: 7 -> 72 VGPRs. With certified walks inside the
// bounce stacks, 64 VGPRs (8 waves) spill in the glass waves that bound a frame: 7 is 2-4 % faster
// on C1-C4 (profiles/r01_v56_ab_occupancy.log), 6 (80 VGPRs) no better.
#if defined(VRT_MIN_WAVES) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_MIN_WAVES is an A/B knob of make variant builds"
#endif
#ifndef VRT_MIN_WAVES  // occupancy A/B builds (make variant); images identical at any value
#define VRT_MIN_WAVES 7
#endif

// The per-frame fields of frame f of a launch (frame batches, KArgs::nframes): its camera, time
// and outputs (the history is read only at alpha != 1, where launches hold one frame)
struct FrameView {
  const float* pv;
  float time;
  uint32_t* cur;
  uint32_t* raw;
};
__device__ __forceinline__ FrameView frame_view(const KArgs& a, uint32_t f) {
  if (f == 0u) return FrameView{a.inv_pv, a.time, a.cur, a.raw};
  const KArgs::FrameB& b = a.fb[f - 1u];
  return FrameView{b.inv_pv, b.time, b.cur, b.raw};
}

// Per-launch constants of the walk context
__device__ __forceinline__ void init_ctx(Ctx& c, const KArgs& a, const uint16_t* __restrict__ vox) {
  c.vox = vox;
  c.ostride = a.ostride;
  c.n = a.n;
  c.p = uint32_t(a.n) + 1u;
  c.fn = a.fn;
  c.max_len = a.max_len;
  c.sky_sy = a.sky_sy;
  c.sun_n = mk(a.sun_n[0], a.sun_n[1], a.sun_n[2]);
  c.sun_rcp = mk(a.sun_rcp[0], a.sun_rcp[1], a.sun_rcp[2]);
  c.time = a.time;
  c.refl_noise = a.refl_noise;
  c.refr_noise = a.refr_noise;
  c.atlas = a.atlas;
  c.atlas_mask = uint32_t(a.atlas_size) - 1u;
  c.atlas_fs = float(a.atlas_size);
  c.atlas_fts = float(a.atlas_tex_size);
#ifdef VRT_CERT_TRACE
  c.tr = false;
#endif
}

// The primary ray of pixel (px, frame row py): vertex stage (voxel.glsl:467-472) evaluated at the
// pixel centre, then stack[0] of main (:430)
// a / d correctly rounded for the vertex stage's divisions: Markstein's division (div_rn) from
// y = RN(1/d) when every operand is far from overflow and underflow (|a|, |d| in [2^-60, 2^60]),
// else the IEEE division; bit-identical either way. Zero numerators take the IEEE division: div_rn
// returns +0 for a = -0 (the residual's zeros cancel to +0), IEEE -0 / d keeps the sign, and a
// -0 component of the direction decides RandomizeDirection's hashes.
__device__ __forceinline__ bool markstein_safe(float x) {
  const float m = __builtin_fabsf(x);
  return m >= 0x1p-60f && m <= 0x1p60f;
}
__device__ __forceinline__ f3 div3_rn(float x, float y, float z, float d) {
  if (markstein_safe(x) && markstein_safe(y) && markstein_safe(z) && markstein_safe(d)) {
    const float r = rcp_newton(d);  // |d| in [2^-60, 2^60]: RN(1/d)
    return mk(div_rn(x, d, r), div_rn(y, d, r), div_rn(z, d, r));
  }
  return mk(x / d, y / d, z / d);
}

__device__ __forceinline__ Ray primary_ray(const KArgs& a, const float* __restrict__ inv_pv, const Ctx& c, int px,
                                           int py) {
  // (2 (p + 0.5)) / W with RN(1/W) from the host: the numerator is in (0, 2W), W <= 32768
  const float ndx = div_rn(2.0f * (float(px) + 0.5f), float(a.width), a.rcp_w) - 1.0f;
  const float ndy = div_rn(2.0f * (float(py) + 0.5f), float(a.height), a.rcp_h) - 1.0f;
  float n4[4], f4[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float base = inv_pv[0 * 4 + i] * ndx + inv_pv[1 * 4 + i] * ndy;
    n4[i] = (base + inv_pv[2 * 4 + i] * -1.0f) + inv_pv[3 * 4 + i] * 1.0f;
    f4[i] = (base + inv_pv[2 * 4 + i] * 1.0f) + inv_pv[3 * 4 + i] * 1.0f;
  }
  const f3 vnear = div3_rn(n4[0], n4[1], n4[2], n4[3]);
  const f3 vdir = div3_rn(f4[0], f4[1], f4[2], f4[3]) - vnear;
  Ray ray;
  ray.pos = mk(vnear.x + c.fn * 0.5f, vnear.y + c.fn * 0.5f, vnear.z + c.fn * 0.5f);
  ray.dir = randomize(normalize3(vdir), vnear, a.ray_noise, c.time);
  ray.len = 0.0f;
  ray.energy = 1.0f;
  ray.voxel = 0;
  ray.rdepth = 0;
  ray.tdepth = 0;
  return ray;
}

// A scratch-stack entry: only reflection rays are stored (exact_pixel), whose medium is air
// (reflection_ray sets voxel 0), with both depths (<= 16) in one word: 9 dwords instead of 11.
struct StackRay {
  f3 pos, dir;
  float len, energy;
  uint32_t depths;
};
__device__ __forceinline__ StackRay pack_stack_ray(const Ray& r) {
  return StackRay{r.pos, r.dir, r.len, r.energy, uint32_t(r.rdepth) | (uint32_t(r.tdepth) << 16)};
}
#if defined(VRT_LDS_STACK) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_LDS_STACK is an A/B knob of make variant builds"
#endif
#ifndef VRT_LDS_STACK  // the bounce stack's bottom entry in LDS (0: every entry in scratch)
#define VRT_LDS_STACK 1
#endif
// The bounce stack's bottom entry of each lane in LDS, component-major (dword j of lane t at
// [j * NL + t]: conflict-free ds_write_b32 / ds_read_b32), the rest in scratch. A pixel whose
// tree holds at most one entry at a time (every C1 pixel: a reflection ray under the first
// refraction ray) then never touches scratch for it.
constexpr int kStackWords = 9;
template <int NL>
__device__ __forceinline__ void lds_stack_put(float* __restrict__ b, const StackRay& e) {
  b[0 * NL] = e.pos.x;
  b[1 * NL] = e.pos.y;
  b[2 * NL] = e.pos.z;
  b[3 * NL] = e.dir.x;
  b[4 * NL] = e.dir.y;
  b[5 * NL] = e.dir.z;
  b[6 * NL] = e.len;
  b[7 * NL] = e.energy;
  b[8 * NL] = __uint_as_float(e.depths);
}
template <int NL>
__device__ __forceinline__ StackRay lds_stack_get(const float* __restrict__ b) {
  return StackRay{mk(b[0 * NL], b[1 * NL], b[2 * NL]), mk(b[3 * NL], b[4 * NL], b[5 * NL]), b[6 * NL],
                  b[7 * NL], __float_as_uint(b[8 * NL])};
}
__device__ __forceinline__ Ray unpack_stack_ray(const StackRay& e) {
  Ray r;
  r.pos = e.pos;
  r.dir = e.dir;
  r.len = e.len;
  r.energy = e.energy;
  r.voxel = 0;
  r.rdepth = int32_t(e.depths & 0xffffu);
  r.tdepth = int32_t(e.depths >> 16);
  return r;
}

#ifdef VRT_STAMPS
// Diagnostic build only: per wave {time after the exact primary trace, after the bounce stacks}
constexpr int kMaxStampWaves3 = 1 << 18;
__device__ unsigned long long g_stamps3[kMaxStampWaves3][2];
#endif

// fragment main (voxel.glsl:425-452) with exact walks. The primary ray (stack[0] of the
// reference) stays in registers; the scratch stack only ever holds secondary rays, so pixels that
// spawn none never touch it. CSH: shadow bits by certified walks from the exact hit points where
// they settle (cert_shadow_exact); CSEC: air-medium secondary rays by certified walks first
// (cert_secondary; on glass-heavy frames their glass hits pay both walks, C1 +19 %: off there).
// Returns whether the pixel ran a bounce stack.
// NL: lanes per workgroup of the LDS stack bottom `lstk` (this lane's word 0; VRT_LDS_STACK).
template <bool STATS, bool TEX, bool CSH = false, bool CSEC = false, int NL = kWgThreads>
__device__ __forceinline__ bool exact_pixel(const KArgs& a, const Ctx& c, Ray ray, f3& color,
                                            Counters& k, uint32_t& steps, uint32_t& flags,
                                            int32_t& hit_vidx, float& hit_len, float* __restrict__ lstk,
                                            float s_init = -1.0f) {
  StackRay stack[kMaxStack - 1 - VRT_LDS_STACK];  // the top entry lives in `ray`, the bottom one in LDS
  const int cap = a.max_refl + a.max_transp + 1;
  int sp = 0;
  const Hit h0 = trace_with_shadow<STATS, TEX, true, CSH>(c, ray, color, k, steps, flags, s_init);
#ifdef VRT_STAMPS
  const uint32_t st_wave = blockIdx.x * kWgWaves + (threadIdx.x >> 6);
  {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (lane_id() == uint32_t(__builtin_amdgcn_readfirstlane(int(lane_id()))) && st_wave < kMaxStampWaves3)
      g_stamps3[st_wave][0] = t;
  }
#endif
  hit_vidx = h0.found ? h0.vidx : -1;
  hit_len = h0.found ? h0.len : 0.0f;
  if (h0.found && mat_id(h0.voxel) == 2) {  // only glass spawns secondary rays (:440-448)
    __builtin_amdgcn_s_setprio(kStackPrio);  // bounce stacks: the longest waves of a frame
    Hit h = h0;
    for (;;) {
      // The sun vector and its reciprocal are opaque per iteration (an empty asm on SGPR copies),
      // so the compiler cannot hoist the per-lane products the loop body forms from them into
      // VGPRs live across the whole loop: those were spilled per lane on loop entry. Scratch
      // 832 -> 720 B per lane, WRITE_SIZE per C3 frame 17.2 -> 14.6 MB (DESIGN.md §6 "HBM writes").
      Ctx lc = c;
      asm volatile("" : "+s"(lc.sun_n.x), "+s"(lc.sun_n.y), "+s"(lc.sun_n.z), "+s"(lc.sun_rcp.x),
                   "+s"(lc.sun_rcp.y), "+s"(lc.sun_rcp.z));
      // The reference pushes the reflection ray, then the refraction ray, then pops the top
      // (:440-448). The ray pushed last is popped at once, so it goes straight to `ray` and only a
      // reflection ray under a refraction ray is written to the scratch stack: same rays in the
      // same order, same STACK_FULL cases (the cap counts the ray held in `ray` as an entry), and
      // about half the scratch writes of a glass tree.
      bool push_r = false, push_t = false;
      if (h.found) {
        const uint32_t m = mat_id(h.voxel);
        const bool pr = mat_reflective(m) && ray.rdepth < a.max_refl;
        const bool pt = mat_transparent(m) && ray.tdepth < a.max_transp && get_color<TEX>(lc, h).w != 1.0f;
        push_r = pr && sp < cap;
        push_t = pt && sp + int(push_r) < cap;
        if ((pr && !push_r) || (pt && !push_t)) flags |= VRT_HIT_FLAG_STACK_FULL;
      }
      if (push_r && push_t) {
        const StackRay e = pack_stack_ray(reflection_ray(lc, ray, h));
        if (VRT_LDS_STACK && sp == 0)
          lds_stack_put<NL>(lstk, e);
        else
          stack[sp - VRT_LDS_STACK] = e;
        ++sp;
        ray = refraction_ray<TEX>(lc, ray, h, k);
      } else if (push_r) {
        ray = reflection_ray(lc, ray, h);
      } else if (push_t) {
        ray = refraction_ray<TEX>(lc, ray, h, k);
      } else {
        if (sp == 0) break;
        --sp;
        ray = unpack_stack_ray(VRT_LDS_STACK && sp == 0 ? lds_stack_get<NL>(lstk) : stack[sp - VRT_LDS_STACK]);
      }
      k.c[VRT_CNT_SECONDARY_RAYS]++;
      if constexpr (CSH && CSEC) {
        bool settled;
        h = march_cert(lc, ray, color, settled, k, steps, flags);
        if (settled) {
          h.found = false;  // a miss or a hit without secondary rays
          continue;
        }
        shade<STATS, TEX, CSH>(lc, ray, h, color, k, steps, flags);
        continue;
      }
      h = trace_with_shadow<STATS, TEX, false, CSH>(lc, ray, color, k, steps, flags);
    }
#ifdef VRT_STAMPS
    {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      if (lane_id() == uint32_t(__builtin_amdgcn_readfirstlane(int(lane_id()))) && st_wave < kMaxStampWaves3)
        g_stamps3[st_wave][1] = t;
    }
#endif
    return true;
  }
  return false;
}

// output of one pixel: float RGBA, or the fused reference post-pass (RGB8 ray-trace store,
// temporal blend, RGB8 store)
__device__ __forceinline__ void store_pixel(const KArgs& a, const FrameView& fv, float4* __restrict__ out,
                                            size_t o, const f3 color) {
  if (fv.cur) {
    const uint32_t rw = pack_rgb8(color.x, color.y, color.z);
    if (fv.raw) fv.raw[o] = rw;
    // u_Alpha = 1 (the slider default): 1 * b/255 + 0 * old stores b back for every byte b and any
    // history (exhaustive, tests/test_temporal_oracle.py), so the history is not read
    fv.cur[o] = a.alpha == 1.0f ? rw : temporal_blend(rw, a.prev[o], a.alpha);
  } else {
    out[o] = make_float4(color.x, color.y, color.z, 1.0f);
  }
}

// One work-item per pixel, 8x8 pixels per wave: the exact path (every launch with hit records or
// counters, textured frames, and colour-only frames when the certified pair below cannot run).
// STATS: this instance writes hit records and/or counters. Without it the per-lane counters,
// step/flag/tie tracking are dead code (~20 VGPRs and a VALU per DDA step freed); the rendering
// arithmetic is the same source in both instances. TEX: textured mode (!_COLOR_ONLY).
// CERT (stats-free colour-only instances): 0 exact walks only, 1 certified walks for the exact
// path's shadow and air-medium secondary rays, 2 also whole pixels first.
// DEFER (certified instances): pixels that need the exact path are not rendered here; their lane
// mask per wave goes to a.defer and exact_pass_kernel renders them compacted (see there).
// The certified pass without the exact path fits 64 VGPRs (8 waves per SIMD) with 8 bytes of
// scratch, but runs faster at 7 (72 VGPRs, no spills): C3 0.0464 -> 0.0447, C4 0.1751 -> 0.1605,
// textured C3 -4 % (profiles/r03_s11, r03_s12); 6 is slower again.
#if (defined(VRT_DEFER_WAVES) || defined(VRT_EXACT_WAVES) || defined(VRT_TPW) || defined(VRT_DIAG_SKIP_EXACT)) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_DEFER_WAVES / VRT_EXACT_WAVES / VRT_TPW are A/B knobs of make variant builds"
#endif
// VRT_TPW (diagnostic): the certified pass's workgroups render VRT_TPW consecutive tiles each, in
// a loop (the multi-tile design of VERDICT r02 #2; record in DESIGN.md §10)
#ifndef VRT_DEFER_WAVES
#define VRT_DEFER_WAVES 7
#endif
#ifndef VRT_EXACT_WAVES
#define VRT_EXACT_WAVES VRT_MIN_WAVES
#endif
// FB: the frame-batch instance (KArgs::nframes > 1: per-frame camera, time and outputs, the frame
// in a deferred entry's top bits); launches of one frame keep the instance without that decode
// (it cost C1 4 %, C3 1 %: profiles/r05_s27)
// TREE (colour-only CERT 2): glass pixels' bounce trees by certified walks (cert_tree), one
// kTreeWords LDS slot per lane.
#if defined(VRT_TREE_WAVES) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_TREE_WAVES is an A/B knob of make variant builds"
#endif
#ifndef VRT_TREE_WAVES  // resident waves per SIMD of the certified pass with certified trees
#define VRT_TREE_WAVES 5
#endif
template <bool STATS, bool TEX, int CERT = 0, bool ORD = false, bool DEFER = false, bool FB = false,
          bool TREE = false>
__global__ void __launch_bounds__(kWgThreads, TREE ? VRT_TREE_WAVES : (DEFER ? VRT_DEFER_WAVES : VRT_MIN_WAVES)) render_kernel(KArgs a, const uint16_t* __restrict__ vox,
                                                     float4* __restrict__ out,
                                                     vrt_hit* __restrict__ hits,
                                                     unsigned long long* __restrict__ counters) {
  // The pixel is re-derived after the trace from wave-uniform SGPRs and a fresh lane id instead
  // of being kept alive across it: at 80 VGPRs the long-lived copies were spilled to scratch by
  // every wave (~1.8 KB/wave of scratch writes, most of the excess WRITE_SIZE over the frame).
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
#ifdef VRT_STAMPS
  const uint32_t wave_lin = blockIdx.x * kWgWaves + wave;
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef VRT_TPW
#pragma nounroll
  for (uint32_t it = 0; it < (DEFER ? uint32_t(VRT_TPW) : 1u); ++it) {
  uint32_t tile = DEFER ? blockIdx.x * uint32_t(VRT_TPW) + it : blockIdx.x;
  if (tile >= a.tiles) break;
#else
  uint32_t tile = blockIdx.x;
#endif
  if constexpr (ORD) {  // heavy-first tile order (a.order): its own instance
    tile = ordered_tile(a, blockIdx.x);
    if (tile == ~0u) return;  // whole workgroup: its tile is rendered by another slot
  }
  tile = __builtin_amdgcn_readfirstlane(tile);
  // frame batches: the tile's frame and its tile within the frame (wave-uniform)
  const uint32_t fr = FB ? uint32_t(__builtin_amdgcn_readfirstlane(int(tile / a.frame_tiles))) : 0u;
  const uint32_t ltile = tile - fr * a.frame_tiles;
  const uint32_t ty = ltile / a.tiles_x, tx = ltile - ty * a.tiles_x;
  const int px = pixel_x(tx, wave, lane_id());
  const int li = pixel_row(ty, wave, lane_id());
  const bool valid = px < a.width && li < a.rows;
  bool heavy = false;  // this lane took the exact path (tile order: the tile runs long next frame)
  bool deferred = false;  // DEFER: this lane's pixel is left to the exact pass

  Counters k;
#pragma unroll
  for (int q = 0; q < VRT_CNT_COUNT; ++q) k.c[q] = 0;

  if (valid) {
    Ctx c;
    init_ctx(c, a, vox);
#ifdef VRT_CERT_TRACE
    c.tr = px == VRT_TRACE_PX && frame_row(a, li) == VRT_TRACE_PY;
#endif
    if constexpr (FB) c.time = frame_view(a, fr).time;
    // one LDS pool: the exact path's axis table and bounce-stack bottom (in-lane instances), and
    // the certified tree's slots (TREE), which are live only before the exact path starts
    constexpr int kAxFloats = DEFER && !TREE ? 0 : kWgThreads * 3 * 4;
    constexpr int kStkFloats = std::max(DEFER || !VRT_LDS_STACK ? 0 : kStackWords * kWgThreads,
                                        TREE ? (kTreeWords - 12) * kWgThreads : 0);
    constexpr int kPool = std::max(kAxFloats + kStkFloats, 4);
    __shared__ float4 lds_pool[kPool / 4];
    c.ax = &lds_pool[threadIdx.x * kAxLane];
#if VRT_DIAG_PHASE == 0
    Ray ray;
    ray.pos = mk(float(px), float(li), 0.0f);
    ray.dir = ray.pos;
    ray.len = 0.0f;
    ray.energy = 1.0f;
    ray.voxel = 0;
    ray.rdepth = ray.tdepth = 0;
#else
    const Ray ray = primary_ray(a, FB ? frame_view(a, fr).pv : a.inv_pv, c, px, frame_row(a, li));
#endif
    k.c[VRT_CNT_PIXELS] = 1;
    k.c[VRT_CNT_PRIMARY_RAYS] = 1;
    uint32_t steps = 0, flags = 0;
    int32_t hit_vidx = -1;
    float hit_len = 0.0f;
    // stats-free colour-only frames: certified primary + shadow walks, the exact path for the
    // rest. cert_pixel starts from its own black colour and writes the result only on success,
    // so no colour value is live (and spilled, 1 KB per wave) across its early exits: C3
    // WRITE_SIZE 41 -> 17 MB per frame at equal speed (profiles/r02_s03). Parking the certified
    // colour in LDS, or storing certified pixels before the exact path and re-deriving the
    // primary ray there, was 4-6 % slower.
    f3 color = mk(0.0f, 0.0f, 0.0f);
    float* tstk = nullptr;
    if constexpr (TREE) {
      static_assert(CERT == 2 && !TEX && !STATS, "certified trees: stats-free colour-only certified instances");
      tstk = reinterpret_cast<float*>(lds_pool) + kAxFloats + threadIdx.x;   // (and c.ax: tree_put)
    }
    float us = -1.0f;  // the primary walk's certified prefix, for the exact path
    const bool need_exact = CERT < 2 || !cert_pixel<TEX, TREE>(c, ray, color, a.max_refl, a.max_transp, tstk, &us);
#ifdef VRT_STAMPS
    const unsigned long long t_cert = __builtin_amdgcn_s_memrealtime();
    const unsigned long long n_exact = __builtin_popcountll(__ballot(need_exact));
    if (lane_id() == 0 && wave_lin < kMaxStampWaves) {
      g_stamps2[wave_lin][0] = t_cert;
      g_stamps2[wave_lin][1] = n_exact;
    }
#endif
    if constexpr (DEFER) {
      deferred = need_exact;
    } else if (need_exact) {
      color = mk(0.0f, 0.0f, 0.0f);
      heavy = true;
      float* lstk = reinterpret_cast<float*>(lds_pool) + kAxFloats;
      (void)exact_pixel<STATS, TEX, CERT >= 1, CERT == 2>(a, c, ray, color, k, steps, flags, hit_vidx,
                                                         hit_len, &lstk[threadIdx.x], STATS ? -1.0f : us);
    }
    const uint32_t l2 = lane_id();
    const size_t o = size_t(pixel_row(ty, wave, l2)) * size_t(a.pitch) + size_t(pixel_x(tx, wave, l2));
    if (STATS && hits) {
      vrt_hit hr;
      hr.voxel_index = hit_vidx;
      hr.ray_length = hit_len;
      hr.steps = steps;
      hr.flags = flags;
      hits[o] = hr;
    }
    // the frame's outputs read here, where they are used (kept live across the walks they were
    // held in registers, and their spills cost the in-lane exact instance 4 %)
    if (!deferred) store_pixel(a, FB ? frame_view(a, fr) : FrameView{a.inv_pv, a.time, a.cur, a.raw}, out, o, color);
  }
  if constexpr (DEFER) {  // the wave's deferred pixels to the exact pass's list: ballot compaction
    const unsigned long long m = __ballot(deferred);
    if (m != 0ull) {
      // segment: the tile's column block of the band (tile column tx * 8 / tiles_x), so that
      // consecutive list entries come from nearby tiles and a sparse batch's rays are alike: C3
      // sparse exact waves 57 -> 49 us median against the 8 XCD classes' every-8th-tile order
      // (profiles/r05_s8 xstamps)
      const uint32_t seg = tx * kOrdClasses / a.tiles_x;
      const uint32_t first = uint32_t(__builtin_ctzll(m));
      const uint32_t cnt = uint32_t(__builtin_popcountll(m));
      // a wave with many deferred pixels (a glass region) keeps them as a chunk of its own, each
      // at its lane (a coherent 8x8 tile of exact work); the others append compactly
      const bool dense = cnt >= kDeferDense;
      uint32_t base = 0;
      if (lane_id() == first)
        base = atomicAdd(a.defer + ((uint32_t(dense) * 2u + a.defer_e) * kOrdClasses + seg) * kOrdCtrStride,
                         dense ? 1u : cnt);
      base = uint32_t(__builtin_amdgcn_readlane(int(base), int(first)));
      uint32_t* list = a.defer + kDeferHdr + seg * a.defer_seg;
      const uint32_t l3 = lane_id();  // the pixel re-derived (not kept live across the walks)
      // frame (3 bits) | band row (13 bits) | column (16 bits): batches need rows < 8192
      const uint32_t id = (fr << 29) | (uint32_t(pixel_row(ty, wave, l3)) << 16) | uint32_t(pixel_x(tx, wave, l3));
      if (dense) {  // chunks fill the segment's region from its end
        list[a.defer_seg - 64u * (base + 1u) + l3] = deferred ? id : ~0u;
      } else if (deferred) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
        list[base + rank] = id;
      }
    }
  }
  if constexpr (ORD) {
    const bool heavy_wave = __ballot(heavy) != 0ull;
    if (lane_id() == 0) order_record(a, tile, heavy_wave);
  }
#ifdef VRT_STAMPS
  {
    // after the tile-order bookkeeping (its atomic's return), so the stamps bracket the whole wave
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    if (lane_id() == 0 && wave_lin < kMaxStampWaves) {
      g_stamps[wave_lin][0] = t_start;
      g_stamps[wave_lin][1] = t_end;
      g_stamps[wave_lin][2] = (unsigned long long)xcc_id() << 32 | hw_id();
    }
  }
#endif
  if (STATS && counters) {
    unsigned long long* slot = counters + size_t(blockIdx.x % kCntReplicas) * VRT_CNT_COUNT;
#pragma unroll
    for (int q = 0; q < VRT_CNT_COUNT; ++q) {
      unsigned long long v = k.c[q];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
      if (lane_id() == 0 && v) atomicAdd(slot + q, v);
    }
  }
#ifdef VRT_TPW
  }
#endif
}

#if (defined(VRT_SPARSE_BATCH) || defined(VRT_SPARSE_BATCH_FAT) || defined(VRT_SPARSE_BATCH_TEX) || defined(VRT_EXACT_PRIO) || \
     defined(VRT_FORCE_FAT)) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_SPARSE_BATCH / VRT_EXACT_PRIO / VRT_FORCE_FAT are A/B knobs of make variant builds"
#endif
// pixels per sparse batch of the exact pass (<= 64): a sparse wave lasts as long as its slowest
// walk and its steps execute the union of its lanes' sampled steps, so smaller batches shorten the
// exact pass's span, which the frame's latency and a short run's drain wait for, at more waves: 32
// with the column-block segments: the driver's 20-frame C3 command 0.0500 -> 0.0464 ms, latency
// 0.123 -> 0.106 ms, 500 frames +0.8 % (C4 +-0, C2 +1 %); 16: 0.0485 / 0.103 / +2.6 %; 8: 0.0479 /
// 0.102 / +6 % (profiles/r05_s10)
#ifndef VRT_SPARSE_BATCH
#define VRT_SPARSE_BATCH 32
#endif
#ifndef VRT_SPARSE_BATCH_TEX  // the same for textured frames: 64 (many more sparse pixels, texel-edge
#define VRT_SPARSE_BATCH_TEX 64  // hits: at 32 the extra waves cost textured C3 0.0572 -> 0.0661 ms, C4
#endif                           // 0.2329 -> 0.2894; profiles/r05_s30)
#ifndef VRT_SPARSE_BATCH_FAT  // the same in the exact pass's 4-wave instance (short bands)
#define VRT_SPARSE_BATCH_FAT 16
#endif
// wave priority of the whole exact pass (0: only its bounce stacks raise it): its few long waves
// share SIMDs with the next frames' certified waves; at 2 their chains issue first (C3 0.0395 ->
// 0.0387 ms per frame, C4 -1 %, the driver's 20-frame run 0.0531 -> 0.0509; 3: C3 0.0389,
// profiles/r04_exact/)
#ifndef VRT_EXACT_PRIO
#define VRT_EXACT_PRIO 2
#endif
#if defined(VRT_FAT_WAVES) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_FAT_WAVES is an A/B knob of make variant builds"
#endif
#ifndef VRT_FAT_WAVES  // resident waves per SIMD of the exact pass's short-band instance
#define VRT_FAT_WAVES 3
#endif
#ifndef VRT_FORCE_FAT  // the short-band exact-pass instance for every colour-only band (A/B only)
#define VRT_FORCE_FAT 0
#endif

// The deferred exact pass: the pixels a certified pass (render_kernel<..., DEFER>) left to it,
// rendered with the exact path 64 to a wave — the certified pass's waves end with their certified
// pixels, and the exact walks that would each have held a sparse wave of them run densely here
// (the north_star's __ballot compaction of live rays). Waves that deferred >= kDeferDense pixels
// (glass regions) left them as a chunk in lane order: one batch each, the same coherent 8x8 tile
// of exact work as in place (textured C3 0.0668 -> 0.0633 ms per frame against compact appends only,
// C2-C4 within +-1.5 %, profiles/r03_s21). The rest
// are batches of 64 list entries over the segments in order. Batches b, b + gridDim.x, ... per
// workgroup.
// Every deferred pixel is rendered exactly once, with the same exact path and epilogue as the
// in-lane fallback, so images are identical. Workgroup 0 zeroes the other counter set for the
// next launch on the stream (none of this launch's kernels reads it).
// WAVES: resident waves per SIMD the instance is built for. 7 (72 VGPRs, ~1 KB of spills per lane)
// for whole frames, where its waves share the CUs with the next frames' certified passes (fewer
// cost 10-30 %, profiles/r03_s25; a spill-free 3-wave instance there: C3 0.0388 -> 0.049 ms per
// frame at 8.7 instead of 17.4 MB of HBM writes, r06_s11); VRT_FAT_WAVES = 3 (no spills: shorter
// exact walks; 168 VGPRs) for colour-only bands of under 4 dispatch rounds and synchronous frames,
// whose frame time is the certified pass plus this pass's latency (a.exact_fat: C4 k = 8 0.0229 ->
// 0.0222, C3 k = 2 0.0275 -> 0.0267 ms at 4 waves, profiles/r03_s67; 3 waves, which no longer
// spill where 4 now do: C4 synchronous frame 0.2125 -> 0.2059 ms, bands of C3/C4 k = 4, 8
// unchanged, r06_s14; textured bands get slower)
// SB: pixels per sparse batch. 64 for whole frames; 16 in the short-band instance,
// whose frame time includes this pass's span: a sparse wave's span is its slowest walk, and a lone
// wave's walks cost the same per step with 16 lanes as with 64 (C4 k = 8 band 0.0222 -> 0.0200 ms,
// exact-pass span 58 -> 49 us; whole frames +1-3 %: more waves, profiles/r04_exact/)
template <bool TEX, int CERT, int WAVES = VRT_EXACT_WAVES, uint32_t SB = VRT_SPARSE_BATCH, bool FB = false>
__global__ void __launch_bounds__(64, WAVES) exact_pass_kernel(KArgs a, const uint16_t* __restrict__ vox,
                                                                     float4* __restrict__ out) {
  const uint32_t* ctr = a.defer;
  if (blockIdx.x == 0 && threadIdx.x < 2u * kOrdClasses) {  // both kinds of the other set, for the next launch
    const uint32_t l = threadIdx.x;
    a.defer[(((l / kOrdClasses) * 2u + (a.defer_e ^ 1u)) * kOrdClasses + l % kOrdClasses) * kOrdCtrStride] = 0u;
  }
#ifdef VRT_DIAG_SKIP_EXACT  // diagnostic bound (wrong images): the frame without its deferred pixels
  return;
#endif
  uint32_t ns[kOrdClasses], nd[kOrdClasses], total_s = 0, total_d = 0;
#pragma unroll
  for (uint32_t q = 0; q < kOrdClasses; ++q) {
    // wave-uniform: kept in SGPRs (as VGPRs they were spilled to scratch by every workgroup,
    // idle ones included, before the early exit below)
    ns[q] = uint32_t(__builtin_amdgcn_readfirstlane(int(ctr[(a.defer_e * kOrdClasses + q) * kOrdCtrStride])));
    nd[q] = uint32_t(__builtin_amdgcn_readfirstlane(int(ctr[((2u + a.defer_e) * kOrdClasses + q) * kOrdCtrStride])));
    total_s += ns[q];
    total_d += nd[q];
  }
  static_assert(SB >= 1 && SB <= 64, "lanes SB.. of a sparse batch idle");
  const uint32_t batches = total_d + (total_s + SB - 1u) / SB;
  if (VRT_EXACT_GRID_ADAPT && a.batches_out && blockIdx.x == 0 && threadIdx.x == 0)
    *a.batches_out = batches;  // for the grid of a later launch on this slot (host-mapped word)
  if (blockIdx.x >= batches) return;  // idle workgroups leave before touching scratch
  if constexpr (VRT_EXACT_PRIO > 0) __builtin_amdgcn_s_setprio(VRT_EXACT_PRIO);
  const uint32_t lane = lane_id();
#ifdef VRT_STAMPS
  const unsigned long long xt0 = __builtin_amdgcn_s_memrealtime();
  uint32_t xlanes = 0;
#endif
  Ctx c;
  init_ctx(c, a, vox);
  __shared__ float4 ax_tab[64 * 3];
  c.ax = &ax_tab[lane * kAxLane];
  for (uint32_t b = blockIdx.x; b < batches; b += gridDim.x) {
    // batch b: dense chunk b (in segment order), else sparse entries [SB (b - total_d), + SB)
    // (sparse batches first measured neutral: C3 0.0386 vs 0.0387 ms, the 20-frame command 0.0453
    // vs 0.0459; profiles/r05_s32)
    const bool dense = b < total_d;
    uint32_t idx = dense ? b : (b - total_d) * SB + lane;
    if (!dense && (lane >= SB || idx >= total_s)) continue;
    uint32_t seg = 0;
#pragma unroll
    for (uint32_t q = 0; q + 1u < kOrdClasses; ++q) {
      const uint32_t nq = dense ? nd[q] : ns[q];
      const bool past = seg == q && idx >= nq;
      idx -= past ? nq : 0u;
      seg += past ? 1u : 0u;
    }
    const uint32_t* list = a.defer + kDeferHdr + seg * a.defer_seg;
    const uint32_t e = dense ? list[a.defer_seg - 64u * (idx + 1u) + lane] : list[idx];
    if (e == ~0u) continue;  // a lane of a dense chunk whose pixel the certified pass settled
    Ray ray;
    if constexpr (FB) {
      const FrameView fv = frame_view(a, e >> 29);
      c.time = fv.time;
      ray = primary_ray(a, fv.pv, c, int(e & 0xFFFFu), frame_row(a, int((e >> 16) & 0x1FFFu)));
    } else {
      ray = primary_ray(a, a.inv_pv, c, int(e & 0xFFFFu), frame_row(a, int(e >> 16)));
    }
    Counters k;
#pragma unroll
    for (int q = 0; q < VRT_CNT_COUNT; ++q) k.c[q] = 0;
    uint32_t steps = 0, flags = 0;
    int32_t hit_vidx = -1;
    float hit_len = 0.0f;
    f3 color = mk(0.0f, 0.0f, 0.0f);
    __shared__ float lstk[VRT_LDS_STACK ? kStackWords * 64 : 1];
    (void)exact_pixel<false, TEX, CERT >= 1, CERT == 2 && !TEX, 64>(a, c, ray, color, k, steps, flags,
                                                                    hit_vidx, hit_len, &lstk[lane]);
    if constexpr (FB) {
      // the pixel and its frame re-derived from e (only e stays live across the exact path)
      uint32_t e2 = e;
      asm volatile("" : "+v"(e2));  // not CSE'd with the decode above (whose results would stay live)
      store_pixel(a, frame_view(a, e2 >> 29), out,
                  size_t((e2 >> 16) & 0x1FFFu) * size_t(a.pitch) + size_t(e2 & 0xFFFFu), color);
    } else {
      store_pixel(a, FrameView{a.inv_pv, a.time, a.cur, a.raw}, out,
                  size_t(e >> 16) * size_t(a.pitch) + size_t(e & 0xFFFFu), color);
    }
#ifdef VRT_STAMPS
    xlanes += uint32_t(__builtin_popcountll(__ballot(true))) | (dense ? 0x10000u : 0u);
#endif
  }
#ifdef VRT_STAMPS
  {
    const unsigned long long xt1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && blockIdx.x < uint32_t(kMaxStampWaves)) {
      g_stamps4[blockIdx.x][0] = xt0;
      g_stamps4[blockIdx.x][1] = xt1;
      g_stamps4[blockIdx.x][2] = (unsigned long long)xcc_id() << 32 | hw_id();
      g_stamps4[blockIdx.x][3] = xlanes;
    }
  }
#endif
}

// Glass and non-empty voxel counts of the canonical volume (vrt_set_certified's automatic mode):
// one wave-reduced atomic pair per wave.
__global__ void __launch_bounds__(256) glass_share_kernel(const uint8_t* __restrict__ vox, uint64_t total,
                                                          unsigned long long* __restrict__ out) {
  unsigned long long g = 0, ne = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < total; i += uint64_t(gridDim.x) * 256) {
    const uint32_t b = vox[i];
    ne += b != 0u ? 1ull : 0ull;
    g += mat_id(b) == 2u ? 1ull : 0ull;
  }
  for (int off = 32; off > 0; off >>= 1) {
    g += __shfl_xor(g, off, 64);
    ne += __shfl_xor(ne, off, 64);
  }
  if ((threadIdx.x & 63u) == 0u) {
    if (g) atomicAdd(out, g);
    if (ne) atomicAdd(out + 1, ne);
  }
}

// Scene builders of main.cpp:218-288 on the device (vrt_build_scene_device): one work-item per
// voxel applies the host builders' writes in their order (csrc/vrt_host.cpp vrt_build_scene);
// `noise` is the n*n terrain heightfield (x + z*n), only read for _TERRAIN.
__global__ void __launch_bounds__(256) build_scene_kernel(uint8_t* __restrict__ vox, int scene,
                                                          uint32_t n, const float* __restrict__ noise) {
  const uint64_t total = uint64_t(n) * n * n;
  const float fs = float(n);
  const uint32_t lo = n / 4, hi = 3 * n / 4, c = n / 2;
  for (uint64_t idx = uint64_t(blockIdx.x) * 256 + threadIdx.x; idx < total;
       idx += uint64_t(gridDim.x) * 256) {
    const uint32_t x = uint32_t(idx % n), y = uint32_t((idx / n) % n), z = uint32_t(idx / (uint64_t(n) * n));
    uint8_t v = 0;
    if (scene == VRT_SCENE_TERRAIN) {  // main.cpp:219-257
      const float h = noise[x + z * n] * fs;
      if (float(int(y)) < h) v = 1;                     // stone column
      if (int(y) == int(h)) v = 3;                      // grass cap
      if (n <= 64) {                                    // glass walls (main.cpp:233)
        if (x == 0 && z >= 2 && z < n - 2 && int(y) >= int(noise[z * n] * fs + 1.0f)) v = 2;
        if (z == n - 4 && x >= 2 && x < n - 1 && int(y) >= int(noise[x * n + n - 4] * fs + 1.0f) &&
            int(y) < int(n) - 4)
          v = 2;
      }
      if (x == n - 1 && z >= 2 && z < n - 2 && int(y) >= int(noise[n - 1 + z * n] * fs + 1.0f) &&
          int(y) < int(n) - 4)
        v = 3;
    } else if (scene == VRT_SCENE_GLASS_CUBE) {  // main.cpp:258-271
      if (x == 0 || x == n - 1 || y == 0 || y == n - 1 || z == 0 || z == n - 1) v = 2;
      if (x == c && y == c && z == c) v = 3;
    } else {  // VRT_SCENE_REFRACTION, main.cpp:272-287
      if (x == c && y == c && z == c) v = 2;
      const bool in_yz = y >= lo && y < hi && z >= lo && z < hi;
      const bool in_xy = x >= lo && x < hi && y >= lo && y < hi;
      const bool in_xz = x >= lo && x < hi && z >= lo && z < hi;
      if (((x == 0 || x == n - 1) && in_yz) || ((z == 0 || z == n - 1) && in_xy) ||
          ((y == 0 || y == n - 1) && in_xz))
        v = 3;
    }
    vox[idx] = v;
  }
}

// Frame assembly of block-cyclic bands (ABI v12; the re-interleave after a gather of the bands to
// one device): band j of k holds the frame's row blocks j, j + k, ... of 2^sh rows, so its row i is
// frame row ((i >> sh) * k + j) * 2^sh + (i & (2^sh - 1)); bands lie band_words words apart. One
// workgroup per frame row copies the row from its band: 16-byte words when VEC (width, band_words
// and frame_pitch multiples of 4 words, 16-byte aligned buffers), else 4-byte words. HBM-bound:
// 8 B of traffic per pixel, no reuse.
template <bool VEC>
__global__ void __launch_bounds__(256) assemble_blocks_kernel(const uint32_t* __restrict__ bands,
                                                              uint64_t band_words, int32_t k, int32_t sh,
                                                              int32_t width, uint32_t* __restrict__ frame,
                                                              uint64_t frame_pitch) {
  const uint32_t y = blockIdx.x;
  const uint32_t m = y >> sh;
  const uint32_t j = m % uint32_t(k), mb = m / uint32_t(k);
  const uint64_t bi = (uint64_t(mb) << sh) + (y & ((1u << sh) - 1u));
  const uint32_t* src = bands + uint64_t(j) * band_words + bi * uint64_t(width);
  uint32_t* dst = frame + uint64_t(y) * frame_pitch;
  if (VEC) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (uint32_t x = threadIdx.x; x < uint32_t(width) / 4u; x += 256u) d4[x] = s4[x];
  } else {
    for (uint32_t x = threadIdx.x; x < uint32_t(width); x += 256u) dst[x] = src[x];
  }
}

// RGB8 wire format of a gathered band (ABI v12): the RGBA8 words' alpha byte is always 255
// (pack_rgb8), so a band crosses xGMI as 3 bytes per pixel — 25 % fewer bytes into rank 0, whose
// ingress bounds the per-frame gather. Four pixels per work-item: one 16-byte load,
// three 4-byte stores (pixels is a multiple of 4).
__global__ void __launch_bounds__(256) pack_rgb8_kernel(const uint4* __restrict__ rgba, uint64_t quads,
                                                        uint32_t* __restrict__ rgb) {
  for (uint64_t q = uint64_t(blockIdx.x) * 256 + threadIdx.x; q < quads; q += uint64_t(gridDim.x) * 256) {
    const uint4 p = rgba[q];
    const uint32_t a = p.x & 0xFFFFFFu, b = p.y & 0xFFFFFFu, c = p.z & 0xFFFFFFu, d = p.w & 0xFFFFFFu;
    // one 12-byte store per work-item (a wave writes 768 contiguous bytes per instruction)
    reinterpret_cast<uint3*>(rgb)[q] = make_uint3(a | (b << 24), (b >> 8) | (c << 16), (c >> 16) | (d << 8));
  }
}

// assemble_blocks_kernel for RGB8 bands (band_px pixels apart, 3 bytes each): each frame row from
// its band, unpacked to RGBA8 words (A = 255); four pixels per work-item (width % 4 == 0)
__global__ void __launch_bounds__(256) assemble_blocks_rgb8_kernel(const uint32_t* __restrict__ bands,
                                                                   uint64_t band_px, int32_t k, int32_t sh,
                                                                   int32_t width, uint4* __restrict__ frame,
                                                                   uint64_t frame_pitch) {
  const uint32_t y = blockIdx.x;
  const uint32_t m = y >> sh;
  const uint32_t j = m % uint32_t(k), mb = m / uint32_t(k);
  const uint64_t bi = (uint64_t(mb) << sh) + (y & ((1u << sh) - 1u));
  const uint32_t* src = bands + (uint64_t(j) * band_px + bi * uint64_t(width)) * 3u / 4u;
  uint4* dst = frame + uint64_t(y) * frame_pitch / 4u;
  for (uint32_t x = threadIdx.x; x < uint32_t(width) / 4u; x += 256u) {
    const uint3 t = reinterpret_cast<const uint3*>(src)[x];  // one 12-byte load (768 B per wave)
    const uint32_t u = t.x, v = t.y, w = t.z;
    dst[x] = make_uint4(0xFF000000u | (u & 0xFFFFFFu), 0xFF000000u | (u >> 24) | ((v & 0xFFFFu) << 8),
                        0xFF000000u | (v >> 16) | ((w & 0xFFu) << 16), 0xFF000000u | (w >> 8));
  }
}

// Diagnostic: RandomizeDirection for n (dir, pos) pairs (vrt_debug_randomize).
__global__ void __launch_bounds__(64) randomize_kernel(const float* __restrict__ dir,
                                                       const float* __restrict__ pos, int n,
                                                       float randomness, float seed,
                                                       float* __restrict__ out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const f3 r = randomize(mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]),
                         mk(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]), randomness, seed);
  out[3 * i] = r.x;
  out[3 * i + 1] = r.y;
  out[3 * i + 2] = r.z;
}

// Sum the counter replicas into `dst` (accumulating) and zero them for the next render.
__global__ void __launch_bounds__(64) reduce_counters_kernel(unsigned long long* __restrict__ rep,
                                                             unsigned long long* __restrict__ dst) {
  const int q = threadIdx.x;
  if (q >= VRT_CNT_COUNT) return;
  unsigned long long s = 0;
  for (int r = 0; r < kCntReplicas; ++r) {
    s += rep[r * VRT_CNT_COUNT + q];
    rep[r * VRT_CNT_COUNT + q] = 0;
  }
  dst[q] += s;
}


// Chebyshev distance field, one separable pass per axis (x, then y, then z), capped at
// kDistCap: out(v) = min(kDistCap, distance to the boundary pseudo-voxels -1 and N on this axis,
// min over |o| < kDistCap of max(|o|, in(v + o e_axis))), where the x pass reads in = 0 for a
// non-empty voxel and kDistCap otherwise. The composition is the exact L-inf distance transform
// (capped), so D(v) >= 1 guarantees an empty box of half-width D-1 around v inside the volume.
__global__ void __launch_bounds__(256) dist_pass_kernel(const uint8_t* __restrict__ in,
                                                        uint8_t* __restrict__ out, uint32_t n,
                                                        int axis, int first) {
  const uint64_t total = uint64_t(n) * n * n;
  const uint64_t stride = axis == 0 ? 1u : (axis == 1 ? uint64_t(n) : uint64_t(n) * n);
  for (uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; q < total;
       q += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t coord = uint32_t((q / stride) % n);
    uint32_t d = min(min(coord + 1u, n - coord), kDistCap);
    for (uint32_t o = 0; o < kDistCap && o < d; ++o) {
      // neighbours at offset -o and +o along the axis
      for (int sgn = -1; sgn <= 1; sgn += 2) {
        if (o == 0 && sgn > 0) break;
        const int64_t cc = int64_t(coord) + sgn * int64_t(o);
        if (cc < 0 || cc >= int64_t(n)) continue;
        const uint8_t v = in[uint64_t(int64_t(q) + (cc - int64_t(coord)) * int64_t(stride))];
        const uint32_t val = first ? (v != 0 ? 0u : kDistCap) : uint32_t(v);
        d = min(d, max(o, val));
      }
    }
    out[q] = uint8_t(d);
  }
}

// Pack into the kernel's padded (N+1)^3 format: voxel | D << 8, plane N repeats plane 0 (GL_REPEAT
// folded into the layout) with D = 0 there (those texels are only read at c == N exactly).
// Single-volume layout (N = 1024).
__global__ void __launch_bounds__(256) pack_volume_kernel(const uint8_t* __restrict__ src,
                                                          const uint8_t* __restrict__ dist,
                                                          uint16_t* __restrict__ dst, uint32_t n) {
  const uint32_t p = n + 1u;
  const uint64_t total = uint64_t(p) * p * p;
  for (uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; q < total;
       q += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t i = uint32_t(q % p), j = uint32_t((q / p) % p), k = uint32_t(q / (uint64_t(p) * p));
    const bool edge = i == n || j == n || k == n;
    const uint32_t si = i == n ? 0u : i, sj = j == n ? 0u : j, sk = k == n ? 0u : k;
    const uint64_t sq = si + (uint64_t(sj) + uint64_t(sk) * n) * n;
    dst[q] = uint16_t(src[sq] | (edge ? 0u : uint32_t(dist[sq]) << 8));
  }
}

// One-sided pass of the octant forward distance along `axis` in direction sg = +-1:
// out(v) = min(kFwdCap, distance to the outside pseudo-voxel ahead (N - c or c + 1),
//              min over 0 <= o of max(o, in(v + sg*o*e_axis))),
// where the first (x) pass reads in = 0 for a non-empty voxel and kFwdCap otherwise. x, then y,
// then z: F(v) = min over non-empty / outside u in v's forward octant of max_a |u_a - v_a| (max
// and min commute through the passes), i.e. the edge of the largest empty in-volume cube
// anchored at v and extending along (sx, sy, sz). max(o, .) >= o, so the scan stops at o = d.
__global__ void __launch_bounds__(256) fwd_pass_kernel(const uint8_t* __restrict__ in,
                                                       uint8_t* __restrict__ out, uint32_t n,
                                                       int axis, int sg, int first) {
  const uint64_t total = uint64_t(n) * n * n;
  const uint64_t stride = axis == 0 ? 1u : (axis == 1 ? uint64_t(n) : uint64_t(n) * n);
  const int64_t step = sg > 0 ? int64_t(stride) : -int64_t(stride);
  for (uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; q < total;
       q += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t coord = uint32_t((q / stride) % n);
    uint32_t d = min(sg > 0 ? n - coord : coord + 1u, kFwdCap);
    // o < d <= the outside distance keeps v + sg*o inside the volume
    for (uint32_t o = 0; o < d; ++o) {
      const uint8_t v = in[uint64_t(int64_t(q) + int64_t(o) * step)];
      const uint32_t val = first ? (v != 0 ? 0u : kFwdCap) : uint32_t(v);
      d = min(d, max(o, val));
    }
    out[q] = uint8_t(d);
  }
}

// Pack octant (sx, sy, sz)'s padded (N+1)^3 volume: voxel | G << 8 with G(v) = F(v - s) - 1
// (0 when v - s is outside or F(v - s) = 0), plane N a copy of plane 0 with G = 0.
__global__ void __launch_bounds__(256) fwd_pack_kernel(const uint8_t* __restrict__ src,
                                                       const uint8_t* __restrict__ fwd,
                                                       uint16_t* __restrict__ dst, uint32_t n,
                                                       int sx, int sy, int sz) {
  const uint32_t p = n + 1u;
  const uint64_t total = uint64_t(p) * p * p;
  for (uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; q < total;
       q += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t i = uint32_t(q % p), j = uint32_t((q / p) % p), k = uint32_t(q / (uint64_t(p) * p));
    const bool edge = i == n || j == n || k == n;
    const uint32_t si = i == n ? 0u : i, sj = j == n ? 0u : j, sk = k == n ? 0u : k;
    const uint64_t sq = si + (uint64_t(sj) + uint64_t(sk) * n) * n;
    uint32_t g = 0;
    const int64_t a = int64_t(i) - sx, b = int64_t(j) - sy, c = int64_t(k) - sz;
    if (!edge && a >= 0 && b >= 0 && c >= 0 && a < int64_t(n) && b < int64_t(n) && c < int64_t(n)) {
      const uint32_t f = fwd[uint64_t(a) + (uint64_t(b) + uint64_t(c) * n) * n];
      g = f > 0u ? f - 1u : 0u;
    }
    dst[q] = uint16_t(src[sq] | (g << 8));
  }
}

}  // namespace vrt

// ------------------------------------------------------------------------------- launches --
// Host wrappers of the kernels above (vrt_internal.h); the C-ABI context is vrt_context.cpp.

namespace vrt {

void launch_render(const KArgs& a, bool stats, const uint16_t* vox, float4* out, vrt_hit* hit,
                   unsigned long long* cnt_rep, hipStream_t s, hipEvent_t ev_begin, hipEvent_t ev_end) {
  const dim3 grid(a.order ? kOrdClasses * a.ord_q + a.tiles : a.tiles);
  // stats-free colour-only frames (vrt_set_certified): certified pixels (a.cert 2), certified
  // exact-path rays only (1: the certified primary's registers would slow glass-heavy frames by
  // ~5 %), exact walks only (0)
  // textured frames: the hit colour needs the exact hit point, so every pixel takes the exact
  // walk; its shadow rays are certified walks where they settle (CERT 1, texture-independent)
  if (a.defer && !stats && a.cert == 2) {
    // certified pass, then the exact pass over the pixels it deferred (no tile order: the
    // certified pass has no long waves)
#ifdef VRT_TPW
    const dim3 g1((a.tiles + VRT_TPW - 1) / VRT_TPW), g2(std::max(64u, a.tiles * uint32_t(kWgWaves) / (a.textured ? kDeferGridDiv : kDeferGridDivColor)));
#else
    const dim3 g1(a.tiles),
        g2(a.exact_grid ? a.exact_grid
                        : std::max(64u, a.tiles * uint32_t(kWgWaves) / (a.textured ? kDeferGridDiv : kDeferGridDivColor)));
#endif
    // frame batches (a.nframes > 1): their own instances
    const bool fb = a.nframes > 1;
    auto k1 = a.textured ? (fb ? render_kernel<false, true, 2, false, true, true> : render_kernel<false, true, 2, false, true>)
              : a.tree   ? (fb ? render_kernel<false, false, 2, false, true, true, true>
                               : render_kernel<false, false, 2, false, true, false, true>)
                         : (fb ? render_kernel<false, false, 2, false, true, true> : render_kernel<false, false, 2, false, true>);
    auto k2 = a.textured ? (fb ? exact_pass_kernel<true, 1, VRT_EXACT_WAVES, VRT_SPARSE_BATCH_TEX, true>
                               : exact_pass_kernel<true, 1, VRT_EXACT_WAVES, VRT_SPARSE_BATCH_TEX>)
                         : ((a.exact_fat || VRT_FORCE_FAT)
                                ? (fb ? exact_pass_kernel<false, 2, VRT_FAT_WAVES, VRT_SPARSE_BATCH_FAT, true>
                                      : exact_pass_kernel<false, 2, VRT_FAT_WAVES, VRT_SPARSE_BATCH_FAT>)
                                : (fb ? exact_pass_kernel<false, 2, VRT_EXACT_WAVES, VRT_SPARSE_BATCH, true>
                                      : exact_pass_kernel<false, 2>));
    if (ev_begin)
      hipExtLaunchKernelGGL(k1, g1, dim3(kWgThreads), 0, s, ev_begin, nullptr, 0, a, vox, out, hit, cnt_rep);
    else
      hipLaunchKernelGGL(k1, g1, dim3(kWgThreads), 0, s, a, vox, out, hit, cnt_rep);
    if (ev_end)
      hipExtLaunchKernelGGL(k2, g2, dim3(64), 0, s, nullptr, ev_end, 0, a, vox, out);
    else
      hipLaunchKernelGGL(k2, g2, dim3(64), 0, s, a, vox, out);
    return;
  }
  auto kern = a.textured ? (stats ? render_kernel<true, true>
                            : a.nframes > 1 ? (a.cert >= 1 ? render_kernel<false, true, 1, false, false, true>
                                                           : render_kernel<false, true, 0, false, false, true>)
                                            : (a.cert >= 1 ? render_kernel<false, true, 1> : render_kernel<false, true>))
                         : (stats ? render_kernel<true, false>
                            : a.nframes > 1
                                ? (a.cert == 2 ? (a.order ? render_kernel<false, false, 2, true, false, true>
                                                          : render_kernel<false, false, 2, false, false, true>)
                                   : a.cert == 1 ? render_kernel<false, false, 1, false, false, true>
                                                 : render_kernel<false, false, 0, false, false, true>)
                                : (a.cert == 2 ? (a.tree ? (a.order ? render_kernel<false, false, 2, true, false, false, true>
                                                                    : render_kernel<false, false, 2, false, false, false, true>)
                                                 : a.order ? render_kernel<false, false, 2, true>
                                                           : render_kernel<false, false, 2>)
                                   : a.cert == 1 ? render_kernel<false, false, 1>
                                                 : render_kernel<false, false, 0>));
  if (ev_begin || ev_end)
    hipExtLaunchKernelGGL(kern, grid, dim3(kWgThreads), 0, s, ev_begin, ev_end, 0, a, vox, out, hit, cnt_rep);
  else
    hipLaunchKernelGGL(kern, grid, dim3(kWgThreads), 0, s, a, vox, out, hit, cnt_rep);
}

void launch_reduce_counters(unsigned long long* rep, unsigned long long* dst, hipStream_t s) {
  hipLaunchKernelGGL(reduce_counters_kernel, dim3(1), dim3(64), 0, s, rep, dst);
}

void launch_volume_passes(const uint8_t* vox, uint8_t* tmp, uint16_t* packed, uint32_t n,
                          int octants, hipStream_t s) {
  const uint64_t vol = uint64_t(n) * n * n, pvol = uint64_t(n + 1) * (n + 1) * (n + 1);
  const unsigned b1 = unsigned(std::min<uint64_t>((vol + 255) / 256, 16384));
  const unsigned b2 = unsigned(std::min<uint64_t>((pvol + 255) / 256, 16384));
  uint8_t* da = tmp;
  uint8_t* db = tmp + vol;
  if (octants == 8) {
    // octant forward distances: 2 x passes, 4 y passes, 8 z passes + packs (x -> y -> z nesting)
    uint8_t* dc = tmp + 2 * vol;
    for (int sx = 1; sx >= -1; sx -= 2) {
      hipLaunchKernelGGL(fwd_pass_kernel, dim3(b1), dim3(256), 0, s, vox, da, n, 0, sx, 1);
      for (int sy = 1; sy >= -1; sy -= 2) {
        hipLaunchKernelGGL(fwd_pass_kernel, dim3(b1), dim3(256), 0, s, da, db, n, 1, sy, 0);
        for (int sz = 1; sz >= -1; sz -= 2) {
          hipLaunchKernelGGL(fwd_pass_kernel, dim3(b1), dim3(256), 0, s, db, dc, n, 2, sz, 0);
          const int o = (sx < 0 ? 1 : 0) | (sy < 0 ? 2 : 0) | (sz < 0 ? 4 : 0);
          hipLaunchKernelGGL(fwd_pack_kernel, dim3(b2), dim3(256), 0, s, vox, dc,
                             packed + size_t(o) * pvol, n, sx, sy, sz);
        }
      }
    }
  } else {
    hipLaunchKernelGGL(dist_pass_kernel, dim3(b1), dim3(256), 0, s, vox, da, n, 0, 1);
    hipLaunchKernelGGL(dist_pass_kernel, dim3(b1), dim3(256), 0, s, da, db, n, 1, 0);
    hipLaunchKernelGGL(dist_pass_kernel, dim3(b1), dim3(256), 0, s, db, da, n, 2, 0);
    hipLaunchKernelGGL(pack_volume_kernel, dim3(b2), dim3(256), 0, s, vox, da, packed, n);
  }
}

void launch_glass_share(const uint8_t* vox, uint64_t total, unsigned long long* out, hipStream_t s) {
  const unsigned b = unsigned(std::min<uint64_t>((total + 255) / 256, 16384));
  hipLaunchKernelGGL(glass_share_kernel, dim3(b), dim3(256), 0, s, vox, total, out);
}

void launch_build_scene(uint8_t* vox, int scene, uint32_t n, const float* noise, hipStream_t s) {
  const uint64_t vol = uint64_t(n) * n * n;
  const unsigned blocks = unsigned(std::min<uint64_t>((vol + 255) / 256, 16384));
  hipLaunchKernelGGL(build_scene_kernel, dim3(blocks), dim3(256), 0, s, vox, scene, n, noise);
}

void launch_assemble_blocks(const uint32_t* bands, uint64_t band_words, int32_t k, int32_t sh, int32_t width,
                            int32_t height, uint32_t* frame, uint64_t frame_pitch, hipStream_t s) {
  if (height <= 0 || width <= 0) return;
  const bool vec = width % 4 == 0 && band_words % 4 == 0 && frame_pitch % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(bands) & 15u) == 0 && (reinterpret_cast<uintptr_t>(frame) & 15u) == 0;
  if (vec)
    hipLaunchKernelGGL(assemble_blocks_kernel<true>, dim3(uint32_t(height)), dim3(256), 0, s, bands, band_words, k,
                       sh, width, frame, frame_pitch);
  else
    hipLaunchKernelGGL(assemble_blocks_kernel<false>, dim3(uint32_t(height)), dim3(256), 0, s, bands, band_words, k,
                       sh, width, frame, frame_pitch);
}

void launch_pack_rgb8(const uint32_t* rgba, uint64_t pixels, uint8_t* rgb, hipStream_t s) {
  const uint64_t quads = pixels / 4u;
  if (quads == 0) return;
  const unsigned blocks = unsigned(std::min<uint64_t>((quads + 255) / 256, 16384));
  hipLaunchKernelGGL(pack_rgb8_kernel, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const uint4*>(rgba), quads,
                     reinterpret_cast<uint32_t*>(rgb));
}

void launch_assemble_blocks_rgb8(const uint8_t* bands, uint64_t band_px, int32_t k, int32_t sh, int32_t width,
                                 int32_t height, uint32_t* frame, uint64_t frame_pitch, hipStream_t s) {
  if (height <= 0 || width <= 0) return;
  hipLaunchKernelGGL(assemble_blocks_rgb8_kernel, dim3(uint32_t(height)), dim3(256), 0, s,
                     reinterpret_cast<const uint32_t*>(bands), band_px, k, sh, width, reinterpret_cast<uint4*>(frame),
                     frame_pitch);
}

// Diagnostic (vrt_debug_fast_math): every float bit pattern, rcp_newton against the IEEE
// division. out: {patterns with rcp_rn_ok, their mismatches, mismatches of normal-range patterns
// with an all-ones significand, mismatches of the other (non-NaN) patterns, the first mismatching
// pattern with rcp_rn_ok (or ~0); then sqrt_fix against the IEEE square root: positive patterns
// with sqrt_fix_ok, their mismatches}
__global__ void fast_math_check_kernel(unsigned long long* out) {
  const uint64_t per = 256;
  const uint64_t base = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) * per;
  uint32_t ok = 0, bad_ok = 0, bad_ones = 0, bad_other = 0, sq_ok = 0, sq_bad = 0;
  for (uint64_t i = 0; i < per; ++i) {
    const uint32_t u = uint32_t(base + i);
    const float d = __uint_as_float(u);
    const uint32_t ex = (u >> 23) & 0xFFu;
    const bool in_range = ex >= 2u && ex <= 252u;
    const bool fine = rcp_rn_ok(d);
    const bool same = __float_as_uint(rcp_newton(d)) == __float_as_uint(1.0f / d);
    ok += fine ? 1u : 0u;
    if (sqrt_fix_ok(d) && d > 0.0f) {
      ++sq_ok;
      if (__float_as_uint(sqrt_fix(d)) != __float_as_uint(__builtin_sqrtf(d))) ++sq_bad;
    }
    if (!same && !(d != d)) {
      if (fine) {
        ++bad_ok;
        atomicMin(&out[4], (unsigned long long)u);
      } else if (in_range) {
        ++bad_ones;
      } else {
        ++bad_other;
      }
    }
  }
  atomicAdd(&out[0], (unsigned long long)ok);
  atomicAdd(&out[1], (unsigned long long)bad_ok);
  atomicAdd(&out[2], (unsigned long long)bad_ones);
  atomicAdd(&out[3], (unsigned long long)bad_other);
  atomicAdd(&out[5], (unsigned long long)sq_ok);
  atomicAdd(&out[6], (unsigned long long)sq_bad);
}

int run_fast_math_check(unsigned long long* host_out) {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, 7 * sizeof(unsigned long long)) != hipSuccess) return VRT_ERR_OOM;
  const unsigned long long init[7] = {0, 0, 0, 0, ~0ull, 0, 0};
  hipError_t e = hipMemcpy(d, init, sizeof(init), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    // 2^32 patterns: 2^24 threads of 256 patterns each
    hipLaunchKernelGGL(fast_math_check_kernel, dim3(1u << 16), dim3(256), 0, nullptr, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(host_out, d, sizeof(init), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  return e == hipSuccess ? VRT_OK : VRT_ERR_DEVICE;
}

void launch_randomize(const float* dir, const float* pos, int n, float randomness, float seed,
                      float* out, hipStream_t s) {
  hipLaunchKernelGGL(randomize_kernel, dim3((n + 63) / 64), dim3(64), 0, s, dir, pos, n,
                     randomness, seed, out);
}

#ifdef VRT_CERT_DIAG
// diagnostic build only: read and reset the certified-walk outcome counts (16 x u64)
int debug_cert_diag(uint64_t* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cert_diag), 32 * 8) != hipSuccess) return VRT_ERR_DEVICE;
  static const uint64_t zero[32] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_cert_diag), zero, 32 * 8) == hipSuccess ? VRT_OK : VRT_ERR_DEVICE;
}
#endif

}  // namespace vrt

#ifdef VRT_STAMPS
extern "C" {
// diagnostic build only: copy the per-wave stamps of the last render (count = 3 x waves)
int vrt_debug_stamps(uint64_t* out, uint64_t count) {
  if (!out || count > 3ull * vrt::kMaxStampWaves) return VRT_ERR_INVALID;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(vrt::g_stamps), count * 8) == hipSuccess ? VRT_OK
                                                                                     : VRT_ERR_DEVICE;
}
int vrt_debug_stamps2(uint64_t* out, uint64_t count) {
  if (!out || count > 2ull * vrt::kMaxStampWaves) return VRT_ERR_INVALID;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(vrt::g_stamps2), count * 8) == hipSuccess ? VRT_OK
                                                                                     : VRT_ERR_DEVICE;
}
int vrt_debug_stamps4(uint64_t* out, uint64_t count) {
  if (!out || count > 4ull * vrt::kMaxStampWaves) return VRT_ERR_INVALID;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(vrt::g_stamps4), count * 8) == hipSuccess ? VRT_OK
                                                                                     : VRT_ERR_DEVICE;
}
int vrt_debug_stamps3(uint64_t* out, uint64_t count) {
  if (!out || count > 2ull * vrt::kMaxStampWaves) return VRT_ERR_INVALID;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(vrt::g_stamps3), count * 8) == hipSuccess ? VRT_OK
                                                                                     : VRT_ERR_DEVICE;
}
#ifdef VRT_CERT_DIAG
int vrt_debug_cert_diag(uint64_t* out) { return out ? vrt::debug_cert_diag(out) : VRT_ERR_INVALID; }
#endif
}  // extern "C"
#elif defined(VRT_CERT_DIAG)
extern "C" int vrt_debug_cert_diag(uint64_t* out) { return out ? vrt::debug_cert_diag(out) : VRT_ERR_INVALID; }
#endif
#ifdef VRT_CERT_TRACE
// diagnostic build: the traced pixel's records (1024 x 8 floats) and their count; resets them
extern "C" int vrt_debug_cert_trace(float* out, uint32_t* count) {
  if (hipDeviceSynchronize() != hipSuccess) return VRT_ERR_DEVICE;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vrt::g_ctrace), 1024 * 8 * 4) != hipSuccess) return VRT_ERR_DEVICE;
  if (hipMemcpyFromSymbol(count, HIP_SYMBOL(vrt::g_ctrace_n), 4) != hipSuccess) return VRT_ERR_DEVICE;
  const uint32_t z = 0;
  return hipMemcpyToSymbol(HIP_SYMBOL(vrt::g_ctrace_n), &z, 4) == hipSuccess ? VRT_OK : VRT_ERR_DEVICE;
}
#endif
