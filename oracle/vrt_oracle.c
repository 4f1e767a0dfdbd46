/*
 * oracle/vrt_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + reported CPU baseline).
 *
 * Scalar C restatement of the reference's per-pixel ray tracer, res/shaders/voxel.glsl, line by
 * line, plus its host-side inputs from src/main.cpp. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product (voxelraytracer_amd/) never
 * does.
 *
 * Parity status: the reference cannot be executed here (GLSL 4.50 needs a GL context; the host
 * needs the un-vendored Greet engine; see DESIGN.md "Oracle"). It ships no tests, golden vectors
 * or fixtures. This restatement is pinned by (1) known-answer tests derived by hand from the
 * GLSL formulas (hash, DDA on hand-built volumes, refract/TIR) and (2) an independent NumPy
 * float32 restatement (oracle/numpy_oracle.py) on small configs. Against the reference itself
 * parity is UNPINNED.
 *
 * GLSL semantics pinned here (the HIP kernel uses the same):
 *   normalize(v) = v * (1/sqrt(x*x+y*y+z*z)), dot left to right, no FMA (-ffp-contract=off)
 *   reflect(I,N) = I - (2*dot(N,I))*N ; refract per the GLSL spec, TIR -> vec3(0)
 *   mix(x,y,a) = x*(1-a) + y*a ; pow(x,y) = exp2(y*log2(x)) ; max = fmaxf ; min(x,y) = y<x?y:x
 *   sign(+-0) = 0 ; IEEE division (±inf on ±0)
 *   texture(): NEAREST + GL_REPEAT on coord/N, i.e. floor(c) mod N for c in [0,N]; NaN -> 0
 *   intersectionAxis[3] (y+z tie) -> clamped to row 2, counted in VRT_CNT_TIE3
 *   every march is cut after VRT_MAX_STEPS iterations (the GLSL would spin), counted
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/vrt.h"

#define EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------ GLSL vector helpers ---- */

typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vdiv(v3 a, v3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline v3 scl(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }   /* v * s */
static inline v3 sclf(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }  /* s * v */
static inline v3 adds(v3 a, float s) { return mk(a.x + s, a.y + s, a.z + s); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline float get(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline void set(v3* a, int i, float f) {
  if (i == 0) a->x = f; else if (i == 1) a->y = f; else a->z = f;
}
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 normalize(v3 v) {
  float inv = 1.0f / sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
  return scl(v, inv);
}
static inline float gsign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
static inline v3 sign3(v3 v) { return mk(gsign(v.x), gsign(v.y), gsign(v.z)); }
static inline float gmin(float x, float y) { return y < x ? y : x; }
static inline float gmax(float x, float y) { return fmaxf(x, y); }
static inline float gpow(float x, float y) { return exp2f(y * log2f(x)); }
static inline float mixf(float x, float y, float a) { return x * (1.0f - a) + y * a; }
/* reflect(I, N) = I - 2.0 * dot(N, I) * N */
static inline v3 reflect(v3 i, v3 n) { float s = 2.0f * dot(n, i); return sub(i, sclf(s, n)); }
/* refract(I, N, eta) per the GLSL 4.50 spec */
static inline v3 refract(v3 i, v3 n, float eta) {
  float d = dot(n, i);
  float k = 1.0f - eta * eta * (1.0f - d * d);
  if (k < 0.0f) return mk(0.0f, 0.0f, 0.0f);
  float s = eta * d + sqrtf(k);
  return sub(sclf(eta, i), sclf(s, n));
}

static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* -------------------------------------------------------- hash RNG, voxel.glsl:98-140 ---- */

EXPORT uint32_t oracle_hash1(uint32_t x) {           /* voxel.glsl:98-106 */
  x += (x << 10u);
  x ^= (x >> 6u);
  x += (x << 3u);
  x ^= (x >> 11u);
  x += (x << 15u);
  return x;
}
EXPORT uint32_t oracle_hash4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { /* :108-111 */
  return oracle_hash1(a ^ oracle_hash1(b) ^ oracle_hash1(c) ^ oracle_hash1(d));
}
EXPORT float oracle_float_construct(uint32_t m) {    /* :115-125 */
  m &= 0x007FFFFFu;
  m |= 0x3F800000u;
  return bitsf(m) - 1.0f;
}
static inline float rnd4(float x, float y, float z, float w) {   /* Random, :127-130 */
  return oracle_float_construct(oracle_hash4(fbits(x), fbits(y), fbits(z), fbits(w)));
}
/* RandomizeDirection, voxel.glsl:132-140 */
static v3 randomize_direction(v3 dir, v3 pos, float randomness, float seed) {
  v3 p = adds(add(pos, dir), seed);
  float dx = rnd4(p.x, p.y, p.z, 0.0f + seed);
  float dy = rnd4(p.x, p.y, p.z, 0.5f + seed);
  float dz = rnd4(p.x, p.y, p.z, 1.0f + seed);
  v3 r = scl(adds(mk(dx, dy, dz), -0.5f), randomness);
  return normalize(add(dir, r));
}
EXPORT void oracle_randomize_direction(const float dir[3], const float pos[3], float randomness,
                                       float seed, float out[3]) {
  v3 r = randomize_direction(mk(dir[0], dir[1], dir[2]), mk(pos[0], pos[1], pos[2]),
                             randomness, seed);
  out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* ---------------------------------------------------------- materials, voxel.glsl:50-93 */

typedef struct {
  float refractivity;
  int transparent, reflective;
  float diffuse, specularity, exponent;
  float color[4];      /* _COLOR_ONLY */
  int tex_x, tex_y;    /* textured: atlas slot */
} material_t;

static const material_t k_materials[4] = {   /* _COLOR_ONLY table :71-87 */
  {1.0f, 1, 0, 0.0f, 0.0f, 0.0f, {0.0f, 0.0f, 0.0f, 0.0f}, 0, 0},    /* Air   :83 */
  {1.0f, 0, 0, 0.4f, 0.2f, 10.0f, {0.5f, 0.5f, 0.5f, 1.0f}, 0, 0},   /* Stone :84 */
  {1.5f, 1, 1, 1.0f, 1.0f, 1.0f, {0.0f, 0.0f, 0.0f, 0.0f}, 0, 0},    /* Glass :85 */
  {1.0f, 0, 0, 0.4f, 0.2f, 10.0f, {0.05f, 0.5f, 0.1f, 1.0f}, 0, 0},  /* Grass :86 */
};
static const material_t k_materials_tex[4] = {   /* textured table :51-68 */
  {1.0f, 1, 0, 0.0f, 0.0f, 0.0f, {0}, 0, 0},      /* Air   :64 */
  {1.0f, 0, 0, 0.4f, 0.6f, 60.0f, {0}, 0, 0},     /* Stone :65 */
  {1.5f, 1, 1, 1.0f, 1.0f, 0.3f, {0}, 0, 1},      /* Glass :66 */
  {1.0f, 0, 0, 0.4f, 0.4f, 20.0f, {0}, 1, 1},     /* Grass :67 */
};
static const float k_ambient = 0.3f;                            /* :91 */

/* ------------------------------------------------------------------------- context ---- */

typedef struct {
  const uint8_t* vox;
  int n;
  float fn;             /* (float)u_Size */
  int textured;         /* !_COLOR_ONLY */
  const uint8_t* atlas; /* RGBA8, atlas_size^2 texels, row 0 = bottom (GL t = 0) */
  int atlas_size, atlas_tex_size;   /* u_AtlasSize, u_AtlasTextureSize */
  v3 sun;               /* u_SunDir as given */
  float time, ray_noise, refl_noise, refr_noise, max_len;
  int max_refl, max_transp;
  const float* inv_pv;
  int width, height;
} ctx_t;

typedef struct {
  uint64_t c[VRT_CNT_COUNT];
} cnt_t;

typedef struct {
  v3 pos, dir;
  float len, energy;
  uint8_t voxel;
  int rdepth, tdepth;
} ray_t;

typedef struct {
  uint8_t voxel;
  v3 point;
  float len;
  v3 normal;
  int found;
  int32_t vidx;
  int index;            /* intersectionAxis row of the step (tie 3 clamped to 2) */
} isect_t;

/* GetMaterial (:156-160): clamp(int(b/255*256), 0, 3) == min(b, 3) for bytes */
static inline const material_t* material(const ctx_t* c, uint8_t b) {
  return &(c->textured ? k_materials_tex : k_materials)[b > 3 ? 3 : b];
}

/* GetTextureCoordinate (:167-172) on the hit's face plane, intersectionAxis[index][1..2] (:93),
 * then texture(u_TextureUnit, uv) (:178): NEAREST + default REPEAT, i = floor(u * S) mod S
 * (GL 4.5 §8.14.2), a NaN coordinate reads texel 0; RGBA8 texels read as b / 255. */
static void get_color(const ctx_t* c, const isect_t* is, float out[4]) {
  const material_t* m = material(c, is->voxel);
  if (!c->textured) {
    for (int q = 0; q < 4; q++) out[q] = m->color[q];
    return;
  }
  static const int ia[3][3] = {{0, 2, 1}, {1, 0, 2}, {2, 0, 1}};
  const float px = get(is->point, ia[is->index][1]), py = get(is->point, ia[is->index][2]);
  const float fx = px - floorf(px), fy = py - floorf(py);
  const float ts = (float)c->atlas_tex_size, as = (float)c->atlas_size;
  const float tx = ((fx + (float)m->tex_x) * ts) / as;
  const float ty = (((1.0f - fy) + (float)m->tex_y) * ts) / as;
  const float u = tx, v = 1.0f - ty;
  const float su = u * as, sv = v * as;
  const int S = c->atlas_size;
  int i = su == su ? (int)floorf(su) : 0, j = sv == sv ? (int)floorf(sv) : 0;
  i = ((i % S) + S) % S;
  j = ((j % S) + S) % S;
  const uint8_t* t = c->atlas + ((size_t)j * S + i) * 4;
  for (int q = 0; q < 4; q++) out[q] = (float)t[q] / 255.0f;
}

/* GetVoxel (:149-154): bounds test with `>` (not `>=`), then NEAREST/REPEAT texel fetch. */
static inline uint8_t get_voxel(const ctx_t* c, v3 p, int32_t* vidx) {
  if (!(p.x >= 0.0f && p.y >= 0.0f && p.z >= 0.0f && p.x <= c->fn && p.y <= c->fn &&
        p.z <= c->fn)) {
    *vidx = -1;
    return 0;
  }
  int i = (int)floorf(p.x), j = (int)floorf(p.y), k = (int)floorf(p.z);
  if (i >= c->n) i -= c->n;   /* c == N reads texel 0 (GL_REPEAT) */
  if (j >= c->n) j -= c->n;
  if (k >= c->n) k -= c->n;
  int32_t idx = i + j * c->n + k * c->n * c->n;
  *vidx = idx;
  return c->vox[idx];
}

/* TestCube (:248-257) with centre N/2 and size N: the ray leaves when outside and moving away. */
static inline int test_cube(v3 p, v3 d, float fn) {
  float hi = fn * 0.5f + fn / 2.0f, lo = fn * 0.5f - fn / 2.0f;
  return !((p.x > hi && d.x > 0.0f) || (p.x < lo && d.x < 0.0f) || (p.y > hi && d.y > 0.0f) ||
           (p.y < lo && d.y < 0.0f) || (p.z > hi && d.z > 0.0f) || (p.z < lo && d.z < 0.0f));
}

static inline float next_plane1(float d, float p) { return d < 0.0f ? ceilf(p - 1.0f) : floorf(p + 1.0f); }
static inline v3 next_plane(v3 d, v3 p) {
  return mk(next_plane1(d.x, p.x), next_plane1(d.y, p.y), next_plane1(d.z, p.z));
}

/* GetReflectionRay (:203-215) */
static ray_t reflection_ray(const ctx_t* c, const ray_t* ray, const isect_t* is) {
  ray_t r;
  r.voxel = 0;
  r.pos = is->point;
  r.dir = randomize_direction(reflect(ray->dir, is->normal), is->point, c->refl_noise, c->time);
  r.len = is->len;
  r.energy = ray->energy * (1.0f - dot(neg(is->normal), ray->dir));  /* Fresnel :162-165 */
  r.rdepth = ray->rdepth + 1;
  r.tdepth = ray->tdepth;
  return r;
}

/* GetRefractionRay (:217-246) */
static ray_t refraction_ray(const ctx_t* c, const ray_t* ray, const isect_t* is, cnt_t* k) {
  int32_t dummy;
  uint8_t outv = get_voxel(c, add(is->point, scl(is->normal, 0.5f)), &dummy);
  uint8_t inv = get_voxel(c, sub(is->point, scl(is->normal, 0.5f)), &dummy);
  k->c[VRT_CNT_REFRACTION_PROBES]++;
  float eta = material(c, outv)->refractivity / material(c, inv)->refractivity;
  ray_t r;
  r.voxel = is->voxel;
  r.pos = is->point;
  r.dir = refract(normalize(ray->dir), is->normal, eta);
  if (r.dir.x == 0.0f && r.dir.y == 0.0f && r.dir.z == 0.0f) {   /* TIR :229-234 */
    r = reflection_ray(c, ray, is);
    r.voxel = ray->voxel;
    r.energy = ray->energy;
  } else {
    r.dir = randomize_direction(r.dir, r.pos, c->refr_noise, c->time);
    r.energy = ray->energy;
    if (ray->voxel == 0) {   /* :239-240 */
      float col[4];
      get_color(c, is, col);
      r.energy *= 1.0f - col[3];
    }
  }
  r.len = is->len;
  r.rdepth = ray->rdepth;
  r.tdepth = ray->tdepth + 1;
  return r;
}

/* RayMarchShadow (:259-300) */
static int march_shadow(const ctx_t* c, const ray_t* ray, cnt_t* k, uint32_t* steps,
                        uint32_t* flags) {
  float rayLength = ray->len;
  v3 cur = ray->pos;
  v3 t = vdiv(sub(next_plane(ray->dir, cur), ray->pos), ray->dir);
  v3 stepDir = sign3(ray->dir);
  uint32_t it = 0;
  while (rayLength < c->max_len) {
    if (!test_cube(cur, ray->dir, c->fn)) return 0;
    if (it >= VRT_MAX_STEPS) { k->c[VRT_CNT_STEP_CAP]++; *flags |= VRT_HIT_FLAG_STEP_CAP; return 0; }
    it++;
    (*steps)++;
    float tMin = gmin(t.x, gmin(t.y, t.z));
    t = adds(t, -tMin);
    rayLength += tMin;
    cur = add(ray->pos, sclf(rayLength - ray->len, ray->dir));
    int ex = t.x == 0.0f, ey = t.y == 0.0f, ez = t.z == 0.0f;
    v3 eq = mk((float)ex, (float)ey, (float)ez);
    int32_t vidx;
    uint8_t voxel = get_voxel(c, add(cur, vmul(sclf(0.5f, eq), stepDir)), &vidx);
    k->c[VRT_CNT_SHADOW_STEPS]++;
    int index = ey + 2 * ez;
    if (index > 2) { index = 2; k->c[VRT_CNT_TIE3]++; *flags |= VRT_HIT_FLAG_TIE3; }
    if (voxel != 0 && !material(c, voxel)->transparent) return 1;
    float q = ((get(cur, index) + get(stepDir, index)) - get(ray->pos, index)) /
                  get(ray->dir, index) - (rayLength - ray->len);
    set(&t, index, q);
  }
  return 0;
}

/* Debug trace of one pixel's ray tree (oracle_trace_pixel; single-threaded, test tooling only):
 * 24-float records, code 1 = a TraceWithShadow call (the ray as it entered RayMarch and its
 * result), code 10 = an in-volume refraction inside RayMarch (crossing point, new ray). */
static float* g_tr = NULL;
static int g_tr_n = 0, g_tr_cap = 0;
static float* tr_rec(float code) {
  if (!g_tr || g_tr_n >= g_tr_cap) return NULL;
  float* r = g_tr + 24 * g_tr_n++;
  for (int i = 0; i < 24; i++) r[i] = 0.0f;
  r[0] = code;
  return r;
}

/* RayMarch (:302-384). `ray` is inout: in-volume refraction mutates it (:361). */
static isect_t march(const ctx_t* c, ray_t* ray, cnt_t* k, uint32_t* steps, uint32_t* flags) {
  isect_t miss;
  memset(&miss, 0, sizeof miss);
  miss.vidx = -1;
  float rayLength = ray->len;
  v3 cur = ray->pos;
  v3 t = vdiv(sub(next_plane(ray->dir, cur), ray->pos), ray->dir);
  v3 stepDir = sign3(ray->dir);
  uint8_t rayVoxel = ray->voxel;
  int internalReflection = 0;
  uint32_t it = 0;
  while (rayLength < c->max_len) {
    if (!test_cube(cur, ray->dir, c->fn)) return miss;
    if (it >= VRT_MAX_STEPS) { k->c[VRT_CNT_STEP_CAP]++; *flags |= VRT_HIT_FLAG_STEP_CAP; return miss; }
    it++;
    (*steps)++;
    float tMin = gmin(t.x, gmin(t.y, t.z));
    t = adds(t, -tMin);
    rayLength += tMin;
    cur = add(ray->pos, sclf(rayLength - ray->len, ray->dir));
    int ex = t.x == 0.0f, ey = t.y == 0.0f, ez = t.z == 0.0f;
    v3 eq = mk((float)ex, (float)ey, (float)ez);
    int32_t vidx;
    uint8_t voxel = get_voxel(c, add(cur, vmul(sclf(0.5f, eq), stepDir)), &vidx);
    k->c[VRT_CNT_DDA_STEPS]++;
    int index = ey + 2 * ez;
    if (index > 2) { index = 2; k->c[VRT_CNT_TIE3]++; *flags |= VRT_HIT_FLAG_TIE3; }
    v3 normal = mk(0.0f, 0.0f, 0.0f);
    set(&normal, index, -gsign(get(ray->dir, index)));
    if (voxel != 0 && voxel != rayVoxel) {
      isect_t h;
      h.voxel = voxel; h.point = cur; h.len = rayLength; h.normal = normal; h.found = 1;
      h.index = index;
      h.vidx = vidx;
      return h;
    } else if (rayVoxel != 0 && voxel == 0) {   /* leaving a transparent voxel :357-380 */
      isect_t is;
      is.voxel = voxel; is.point = cur; is.len = rayLength; is.normal = normal; is.found = 1;
      is.index = index;
      is.vidx = vidx;
      v3 oldDir = ray->dir;
      *ray = refraction_ray(c, ray, &is, k);
      ray->tdepth--;
      if (ray->voxel == rayVoxel) {
        internalReflection++;
        if (internalReflection > 10) { ray->dir = oldDir; ray->voxel = 0; }
      }
      float* r = tr_rec(10.0f);
      if (r) {
        r[1] = (float)index; r[2] = cur.x; r[3] = cur.y; r[4] = cur.z; r[5] = rayLength;
        r[6] = ray->dir.x; r[7] = ray->dir.y; r[8] = ray->dir.z; r[9] = (float)ray->voxel;
        r[10] = ray->energy; r[11] = (float)it;
      }
      rayVoxel = ray->voxel;
      t = vdiv(sub(next_plane(ray->dir, cur), ray->pos), ray->dir);
      stepDir = sign3(ray->dir);
    }
    float q = ((get(cur, index) + get(stepDir, index)) - get(ray->pos, index)) /
                  get(ray->dir, index) - (rayLength - ray->len);
    set(&t, index, q);
  }
  return miss;
}

/* GetSkyboxColor (:386-393) */
static v3 skybox(const ctx_t* c, const ray_t* ray, v3 color) {
  v3 u = normalize(ray->dir);
  float sun = 10.0f * gpow(dot(normalize(c->sun), u), 400.0f);
  float grad = (u.y + 1.0f) * 0.5f;
  float sy = gmax(c->sun.y, 0.0f);
  v3 sk = mk(gmax(0.0f, sun) * sy, gmax(grad * 0.75f, sun) * sy, gmax(grad, 0.0f) * sy);
  float a = 1.0f - ray->energy;
  return mk(mixf(sk.x, color.x, a), mixf(sk.y, color.y, a), mixf(sk.z, color.z, a));
}

/* TraceWithShadow (:395-423) */
static isect_t trace_with_shadow(const ctx_t* c, ray_t* ray, v3* color, cnt_t* k,
                                 uint32_t* steps, uint32_t* flags) {
  float* tr = tr_rec(1.0f);
  if (tr) {
    tr[9] = ray->pos.x; tr[10] = ray->pos.y; tr[11] = ray->pos.z; tr[12] = ray->dir.x; tr[13] = ray->dir.y;
    tr[14] = ray->dir.z; tr[15] = ray->len; tr[16] = ray->energy; tr[17] = (float)ray->voxel;
    tr[18] = (float)ray->rdepth; tr[19] = (float)ray->tdepth;
  }
  isect_t is = march(c, ray, k, steps, flags);
  if (tr) {
    tr[1] = (float)is.found; tr[2] = (float)is.voxel; tr[3] = (float)is.index; tr[4] = is.point.x;
    tr[5] = is.point.y; tr[6] = is.point.z; tr[7] = is.len;
  }
  if (is.found) {
    ray_t sr;   /* GetShadowRay :191-201 */
    sr.voxel = is.voxel;
    sr.pos = is.point;
    sr.dir = normalize(c->sun);
    sr.len = is.len;
    sr.energy = ray->energy;
    sr.rdepth = 0;
    sr.tdepth = 0;
    k->c[VRT_CNT_SHADOW_RAYS]++;
    int in_shadow = march_shadow(c, &sr, k, steps, flags);
    float brightness;
    const material_t* m = material(c, is.voxel);
    if (in_shadow) {
      brightness = k_ambient;
    } else {
      float diffuse = m->diffuse * gmax(dot(is.normal, sr.dir), 0.0f);
      float specular = m->specularity *
                       gpow(gmax(dot(reflect(sr.dir, is.normal), ray->dir), 0.0f), m->exponent);
      brightness = k_ambient + diffuse + specular;
    }
    /* RayColor :184-188 */
    float e = ray->energy;
    float col[4];
    get_color(c, &is, col);
    float a = col[3];
    color->x = mixf(color->x, col[0] * a * brightness, e);
    color->y = mixf(color->y, col[1] * a * brightness, e);
    color->z = mixf(color->z, col[2] * a * brightness, e);
  } else {
    v3 sk = skybox(c, ray, *color);
    float a = 1.0f - ray->energy;
    *color = mk(mixf(sk.x, color->x, a), mixf(sk.y, color->y, a), mixf(sk.z, color->z, a));
  }
  return is;
}

#define MAX_STACK 17

/* fragment main (:425-452) with the vertex stage (:467-472) evaluated at the pixel centre. */
static void shade_pixel(const ctx_t* c, int px, int py, float* rgba, vrt_hit* hit, cnt_t* k) {
  float ndx = (2.0f * ((float)px + 0.5f)) / (float)c->width - 1.0f;
  float ndy = (2.0f * ((float)py + 0.5f)) / (float)c->height - 1.0f;
  const float* m = c->inv_pv;
  float n4[4], f4[4];
  for (int i = 0; i < 4; i++) {
    n4[i] = ((m[0 * 4 + i] * ndx + m[1 * 4 + i] * ndy) + m[2 * 4 + i] * -1.0f) + m[3 * 4 + i] * 1.0f;
    f4[i] = ((m[0 * 4 + i] * ndx + m[1 * 4 + i] * ndy) + m[2 * 4 + i] * 1.0f) + m[3 * 4 + i] * 1.0f;
  }
  v3 vnear = mk(n4[0] / n4[3], n4[1] / n4[3], n4[2] / n4[3]);
  v3 vdir = sub(mk(f4[0] / f4[3], f4[1] / f4[3], f4[2] / f4[3]), vnear);

  v3 color = mk(0.0f, 0.0f, 0.0f);
  ray_t stack[MAX_STACK];
  int cap = c->max_refl + c->max_transp + 1;
  stack[0].pos = adds(vnear, c->fn * 0.5f);
  stack[0].dir = randomize_direction(normalize(vdir), vnear, c->ray_noise, c->time);
  stack[0].len = 0.0f;
  stack[0].energy = 1.0f;
  stack[0].voxel = 0;
  stack[0].rdepth = 0;
  stack[0].tdepth = 0;
  int sp = 1;
  uint32_t steps = 0, flags = 0;
  int first = 1;
  k->c[VRT_CNT_PIXELS]++;
  k->c[VRT_CNT_PRIMARY_RAYS]++;
  hit->voxel_index = -1;
  hit->ray_length = 0.0f;
  while (sp > 0) {
    ray_t ray = stack[--sp];
    if (!first) k->c[VRT_CNT_SECONDARY_RAYS]++;
    isect_t is = trace_with_shadow(c, &ray, &color, k, &steps, &flags);
    if (first) {
      if (is.found) { hit->voxel_index = is.vidx; hit->ray_length = is.len; }
      first = 0;
    }
    if (is.found) {
      const material_t* mt = material(c, is.voxel);
      if (mt->reflective && ray.rdepth < c->max_refl) {
        if (sp < cap) stack[sp++] = reflection_ray(c, &ray, &is);
        else flags |= VRT_HIT_FLAG_STACK_FULL;
      }
      float col[4];
      if (mt->transparent && ray.tdepth < c->max_transp && (get_color(c, &is, col), col[3] != 1.0f)) {
        if (sp < cap) stack[sp++] = refraction_ray(c, &ray, &is, k);
        else flags |= VRT_HIT_FLAG_STACK_FULL;
      }
    }
  }
  rgba[0] = color.x;
  rgba[1] = color.y;
  rgba[2] = color.z;
  rgba[3] = 1.0f;
  hit->steps = steps;
  hit->flags = flags;
}

/* ------------------------------------------------------------------ threaded driver ---- */

typedef struct {
  const ctx_t* c;
  int row0, rows, row_step;
  float* out;
  vrt_hit* hits;
  int next;            /* atomic row cursor */
  pthread_mutex_t mu;
  cnt_t total;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  cnt_t k;
  memset(&k, 0, sizeof k);
  for (;;) {
    int i = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
    if (i >= j->rows) break;
    int py = j->row0 + i * j->row_step;
    for (int px = 0; px < j->c->width; px++) {
      size_t o = (size_t)i * j->c->width + px;
      vrt_hit h;
      shade_pixel(j->c, px, py, j->out + 4 * o, &h, &k);
      if (j->hits) j->hits[o] = h;
    }
  }
  pthread_mutex_lock(&j->mu);
  for (int q = 0; q < VRT_CNT_COUNT; q++) j->total.c[q] += k.c[q];
  pthread_mutex_unlock(&j->mu);
  return NULL;
}

/* Render rows row0 + i*row_step (i < rows) at full width; same layout contract as
 * vrt_render_rows_async. counters: VRT_CNT_COUNT uint64 (accumulated). Returns 0 or <0. */
EXPORT int oracle_render(const vrt_camera* cam, const uint8_t* vox, int n, const vrt_params* p,
                         int row0, int rows, int row_step, float* out_rgba, vrt_hit* out_hit,
                         uint64_t* counters, int nthreads) {
  if (!cam || !vox || !p || !out_rgba || n <= 0 || rows < 0) return VRT_ERR_INVALID;
  if (!p->color_only && (!p->atlas_rgba || p->atlas_size <= 0 || p->atlas_texture_size <= 0))
    return VRT_ERR_INVALID;
  if (p->max_reflections < 0 || p->max_transparencies < 0 ||
      p->max_reflections + p->max_transparencies + 1 > MAX_STACK)
    return VRT_ERR_UNSUPPORTED;
  ctx_t c;
  c.vox = vox;
  c.n = n;
  c.fn = (float)n;
  c.sun = mk(p->sun_dir[0], p->sun_dir[1], p->sun_dir[2]);
  c.time = p->time;
  c.ray_noise = p->ray_noise;
  c.refl_noise = p->reflection_noise;
  c.refr_noise = p->refraction_noise;
  c.max_len = p->max_ray_length;
  c.max_refl = p->max_reflections;
  c.max_transp = p->max_transparencies;
  c.inv_pv = cam->inv_pv;
  c.textured = !p->color_only;
  c.atlas = p->atlas_rgba;
  c.atlas_size = p->atlas_size;
  c.atlas_tex_size = p->atlas_texture_size;
  c.width = cam->width;
  c.height = cam->height;
  job_t j;
  memset(&j, 0, sizeof j);
  j.c = &c;
  j.row0 = row0;
  j.rows = rows;
  j.row_step = row_step;
  j.out = out_rgba;
  j.hits = out_hit;
  pthread_mutex_init(&j.mu, NULL);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  for (int i = 1; i < nthreads; i++) pthread_create(&th[i], NULL, worker, &j);
  worker(&j);
  for (int i = 1; i < nthreads; i++) pthread_join(th[i], NULL);
  pthread_mutex_destroy(&j.mu);
  if (counters)
    for (int q = 0; q < VRT_CNT_COUNT; q++) counters[q] += j.total.c[q];
  return VRT_OK;
}

/* Debug: the ray tree of pixel (px, frame row py) as 24-float records (see tr_rec), at most cap;
 * returns the record count (<0: error), rgba the pixel's colour. */
EXPORT int oracle_trace_pixel(const vrt_camera* cam, const uint8_t* vox, int n, const vrt_params* p, int px,
                              int py, float* out, int cap, float rgba[4]) {
  if (!cam || !vox || !p || !out || !p->color_only) return VRT_ERR_INVALID;
  ctx_t c;
  memset(&c, 0, sizeof c);
  c.vox = vox;
  c.n = n;
  c.fn = (float)n;
  c.sun = mk(p->sun_dir[0], p->sun_dir[1], p->sun_dir[2]);
  c.time = p->time;
  c.ray_noise = p->ray_noise;
  c.refl_noise = p->reflection_noise;
  c.refr_noise = p->refraction_noise;
  c.max_len = p->max_ray_length;
  c.max_refl = p->max_reflections;
  c.max_transp = p->max_transparencies;
  c.inv_pv = cam->inv_pv;
  c.width = cam->width;
  c.height = cam->height;
  cnt_t k;
  memset(&k, 0, sizeof k);
  vrt_hit h;
  g_tr = out;
  g_tr_n = 0;
  g_tr_cap = cap;
  shade_pixel(&c, px, py, rgba, &h, &k);
  g_tr = NULL;
  return g_tr_n;
}

/* Trace ONE ray through RayMarch (for hand-built DDA known-answer tests). Returns found. */
EXPORT int oracle_march_one(const uint8_t* vox, int n, const float pos[3], const float dir[3],
                            float max_len, int32_t* out_vidx, float* out_len, float out_point[3],
                            float out_normal[3], uint32_t* out_steps) {
  ctx_t c;
  memset(&c, 0, sizeof c);
  c.vox = vox;
  c.n = n;
  c.fn = (float)n;
  c.max_len = max_len;
  c.sun = mk(0.0f, 1.0f, 0.0f);
  cnt_t k;
  memset(&k, 0, sizeof k);
  ray_t r;
  memset(&r, 0, sizeof r);
  r.pos = mk(pos[0], pos[1], pos[2]);
  r.dir = mk(dir[0], dir[1], dir[2]);
  r.energy = 1.0f;
  uint32_t steps = 0, flags = 0;
  isect_t h = march(&c, &r, &k, &steps, &flags);
  *out_vidx = h.found ? h.vidx : -1;
  *out_len = h.len;
  out_point[0] = h.point.x; out_point[1] = h.point.y; out_point[2] = h.point.z;
  out_normal[0] = h.normal.x; out_normal[1] = h.normal.y; out_normal[2] = h.normal.z;
  *out_steps = steps;
  return h.found;
}

EXPORT void oracle_refract(const float i[3], const float nrm[3], float eta, float out[3]) {
  v3 r = refract(mk(i[0], i[1], i[2]), mk(nrm[0], nrm[1], nrm[2]), eta);
  out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* ----------------------------------------------- host inputs restated from src/main.cpp ---- */

/* Terrain heightfield: the build-defined generator of DESIGN.md "Terrain noise" (Greet's
 * Noise::GenNoise is not vendored). Value noise, 5 octaves, lattice spacing n/(4<<octave) (min 1),
 * amplitude persistence^octave, smoothstep-bilinear, in double, mapped to 0.2+0.3*v, rounded to
 * float. */
static uint32_t lattice_hash(uint32_t seed, uint32_t o, uint32_t i, uint32_t j) {
  uint32_t h = seed * 0x9E3779B1u ^ o * 0x85EBCA77u ^ i * 0xC2B2AE3Du ^ j * 0x27D4EB2Fu;
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}
static double lattice(uint32_t seed, int o, int i, int j) {
  return (double)(lattice_hash(seed, (uint32_t)o, (uint32_t)i, (uint32_t)j) >> 8) * (1.0 / 16777216.0);
}
EXPORT int oracle_terrain_noise(int n, uint32_t seed, float* out) {
  const int octaves = 5;
  const double persistence = n <= 32 ? 0.5 : 0.125;   /* main.cpp:185 vs :195 */
  for (int z = 0; z < n; z++) {
    for (int x = 0; x < n; x++) {
      double sum = 0.0, total = 0.0, amp = 1.0;
      for (int o = 0; o < octaves; o++) {
        int step = n / (4 << o);
        if (step < 1) step = 1;
        int i0 = x / step, j0 = z / step;
        double fx = (double)(x - i0 * step) / (double)step;
        double fz = (double)(z - j0 * step) / (double)step;
        fx = fx * fx * (3.0 - 2.0 * fx);
        fz = fz * fz * (3.0 - 2.0 * fz);
        double a = lattice(seed, o, i0, j0), b = lattice(seed, o, i0 + 1, j0);
        double cc = lattice(seed, o, i0, j0 + 1), d = lattice(seed, o, i0 + 1, j0 + 1);
        double top = a + (b - a) * fx, bot = cc + (d - cc) * fx;
        sum += amp * (top + (bot - top) * fz);
        total += amp;
        amp *= persistence;
      }
      float v = (float)(0.2 + 0.3 * (sum / total));
      if (v >= 1.0f) v = 0x1.fffffep-1f;
      if (v < 0.0f) v = 0.0f;
      out[x + z * n] = v;
    }
  }
  return 0;
}

/* main.cpp:218-288 */
EXPORT int oracle_build_scene(int scene, int n, uint32_t seed, uint8_t* data) {
  if (n < 8 || n > 1024) return VRT_ERR_INVALID;
  const unsigned size = (unsigned)n;
  const size_t s2 = (size_t)size * size;
  memset(data, 0, s2 * size);
  if (scene == VRT_SCENE_TERRAIN) {
    float* noise = (float*)malloc(sizeof(float) * s2);
    oracle_terrain_noise(n, seed, noise);
    for (unsigned z = 0; z < size; z++) {
      for (unsigned x = 0; x < size; x++) {
        for (int y = 0; (float)y < noise[x + z * size] * (float)size; y++)
          data[x + (size_t)y * size + z * s2] = 1;
        int grassLevel = (int)(noise[x + z * size] * (float)size);
        data[x + (size_t)grassLevel * size + z * s2] = 3;
      }
    }
    if (size <= 64) {
      for (unsigned z = 2; z < size - 2; z++)
        for (int y = (int)(noise[z * size] * (float)size + 1.0f); y < (int)size; y++)
          data[(size_t)y * size + z * s2] = 2;
      for (unsigned x = 2; x < size - 1; x++)
        for (int y = (int)(noise[x * size + size - 4] * (float)size + 1.0f); y < (int)size - 4; y++)
          data[x + (size_t)y * size + (size - 4) * s2] = 2;
    }
    for (unsigned z = 2; z < size - 2; z++)
      for (int y = (int)(noise[size - 1 + z * size] * (float)size + 1.0f); y < (int)size - 4; y++)
        data[size - 1 + (size_t)y * size + z * s2] = 3;
    free(noise);
  } else if (scene == VRT_SCENE_GLASS_CUBE) {
    for (size_t i = 0; i < size; i++) {
      for (size_t j = 0; j < size; j++) {
        data[size - 1 + i * size + j * s2] = 2;
        data[i * size + j * s2] = 2;
        data[i + j * size + (size - 1) * s2] = 2;
        data[i + j * size] = 2;
        data[i + (size - 1) * size + j * s2] = 2;
        data[i + j * s2] = 2;
      }
    }
    data[size / 2 + size / 2 * size + size / 2 * s2] = 3;
  } else if (scene == VRT_SCENE_REFRACTION) {
    data[size / 2 + size / 2 * size + size / 2 * s2] = 2;
    for (size_t i = size / 4; i < 3 * size / 4; i++) {
      for (size_t j = size / 4; j < 3 * size / 4; j++) {
        data[size - 1 + i * size + j * s2] = 3;
        data[i * size + j * s2] = 3;
        data[i + j * size + (size - 1) * s2] = 3;
        data[i + j * size] = 3;
        data[i + (size - 1) * size + j * s2] = 3;
        data[i + j * s2] = 3;
      }
    }
  } else {
    return VRT_ERR_INVALID;
  }
  return VRT_OK;
}

/* ---- Temporal filter and RGB8 framebuffer store ----
 * The ray-trace FBO and the two temporal FBOs are RGB8 textures (FrameBuffer.cpp:8, internal
 * format RGB). Writing the shader's vec4 colour stores each of R, G, B as a normalized 8-bit value;
 * GL's float -> UNORM conversion clamps to [0,1], scales by 255 and rounds to nearest. The tie
 * rule (x.5) and NaN handling are implementation-defined in GL; this restatement pins ties to
 * even (rintf) and NaN to 0 (fmaxf drops it). Sampling an RGB8 texel returns b / 255.
 * temporal.glsl:18: color = u_Alpha * newColor + (1 - u_Alpha) * averageColor, stored to the
 * current RGB8 FBO (main.cpp:363-377), then current and last swap (main.cpp:391). Pixels are
 * RGBA8 words here, R in the low byte, A = 255 (the FBOs have no alpha channel).
 */
static inline uint8_t unorm8(float f) {
  const float c = fminf(fmaxf(f, 0.0f), 1.0f);
  return (uint8_t)rintf(c * 255.0f);
}
static inline float unorm8_read(uint8_t b) { return (float)b / 255.0f; }

EXPORT void oracle_temporal(const float* rgba, const uint8_t* prev_rgba8, float alpha,
                            uint8_t* raw_rgba8, uint8_t* cur_rgba8, uint64_t npix) {
  const float one_minus = 1.0f - alpha;
  for (uint64_t i = 0; i < npix; i++) {
    for (int ch = 0; ch < 3; ch++) {
      const uint8_t raw = unorm8(rgba[i * 4 + ch]);
      if (raw_rgba8) raw_rgba8[i * 4 + ch] = raw;
      const float nw = unorm8_read(raw);
      const float old = unorm8_read(prev_rgba8[i * 4 + ch]);
      cur_rgba8[i * 4 + ch] = unorm8(alpha * nw + one_minus * old);
    }
    if (raw_rgba8) raw_rgba8[i * 4 + 3] = 255;
    cur_rgba8[i * 4 + 3] = 255;
  }
}

/* the same blend from already-quantised new pixels (raw RGBA8), for checking the device's
 * epilogue bit-exactly on its own raw output */
EXPORT void oracle_temporal_from_raw(const uint8_t* raw_rgba8, const uint8_t* prev_rgba8, float alpha,
                                     uint8_t* cur_rgba8, uint64_t npix) {
  const float one_minus = 1.0f - alpha;
  for (uint64_t i = 0; i < npix; i++) {
    for (int ch = 0; ch < 3; ch++) {
      const float nw = unorm8_read(raw_rgba8[i * 4 + ch]);
      const float old = unorm8_read(prev_rgba8[i * 4 + ch]);
      cur_rgba8[i * 4 + ch] = unorm8(alpha * nw + one_minus * old);
    }
    cur_rgba8[i * 4 + 3] = 255;
  }
}

/* GetColor for one hit (known-answer tests of the textured path) */
EXPORT void oracle_get_color(const uint8_t* atlas, int atlas_size, int atlas_tex_size, int textured,
                             uint8_t voxel, const float point[3], int index, float out[4]) {
  ctx_t c;
  memset(&c, 0, sizeof c);
  c.textured = textured;
  c.atlas = atlas;
  c.atlas_size = atlas_size;
  c.atlas_tex_size = atlas_tex_size;
  isect_t is;
  memset(&is, 0, sizeof is);
  is.voxel = voxel;
  is.point = mk(point[0], point[1], point[2]);
  is.index = index;
  get_color(&c, &is, out);
}
