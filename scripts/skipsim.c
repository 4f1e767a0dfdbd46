/* Skip-window simulator (analysis tool, not product, not oracle): replays the primary and shadow
 * DDA walks of the reference (voxel.glsl:259-384; secondary rays omitted) on the CPU and counts,
 * per empty-space scheme, how many steps must sample the volume and how many 8x8 wave-steps
 * contain at least one sampling lane (lockstep approximation: a wave's k-th step samples if any
 * lane's k-th step does, per walk phase).
 *   scheme 0: centred Chebyshev distance D (the kernel today: box [v-D+1, v+D-1]^3)
 *   scheme 1: octant distance F (largest empty cube [v, v+(F-1)s]^3 in the ray's direction octant)
 *   scheme 2: guarded octant distance F' = F(v - s) - 1 (the cube also covers one voxel behind v on
 *             every axis, so samples that rounding puts just behind an entry face stay covered)
 *   scheme 3: F if the behind slabs {v - s_a e_a + {0, s_b} x {0, s_c}} are empty, else F' 
 * Build: gcc -O2 -ffp-contract=off -fopenmp -shared -fPIC -o build/skipsim.so scripts/skipsim.c
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NS 4
typedef struct { float x, y, z; } v3;

static int N;
static const uint8_t* VOX;
static uint8_t* DC;     /* centred distance, cap */
static uint8_t* FO[8];  /* octant distance, cap */

static inline int occ(int i, int j, int k) {
  if (i < 0 || j < 0 || k < 0 || i >= N || j >= N || k >= N) return 1;
  return VOX[i + (size_t)N * (j + (size_t)N * k)] != 0;
}

void sim_build(const uint8_t* vox, int n, int capc, int capo) {
  N = n;
  VOX = vox;
  size_t tot = (size_t)n * n * n;
  DC = malloc(tot);
  /* centred Chebyshev (L-inf) distance to the nearest occupied voxel or the outside, separable:
   * 1D along x, then min over y of max(|dy|, .), then over z */
  int* dx = malloc(tot * sizeof(int));
  int* dy = malloc(tot * sizeof(int));
#pragma omp parallel for
  for (int k = 0; k < n; k++)
    for (int j = 0; j < n; j++)
      for (int i = 0; i < n; i++) {
        int best = i + 1 < n - i ? i + 1 : n - i;
        for (int a = 0; a < n; a++)
          if (VOX[a + (size_t)n * (j + (size_t)n * k)] && abs(a - i) < best) best = abs(a - i);
        dx[i + (size_t)n * (j + (size_t)n * k)] = best;
      }
#pragma omp parallel for
  for (int k = 0; k < n; k++)
    for (int j = 0; j < n; j++)
      for (int i = 0; i < n; i++) {
        int best = j + 1 < n - j ? j + 1 : n - j;
        for (int b = 0; b < n; b++) {
          int v = dx[i + (size_t)n * (b + (size_t)n * k)], e = abs(b - j);
          int m = v > e ? v : e;
          if (m < best) best = m;
        }
        dy[i + (size_t)n * (j + (size_t)n * k)] = best;
      }
#pragma omp parallel for
  for (int k = 0; k < n; k++)
    for (int j = 0; j < n; j++)
      for (int i = 0; i < n; i++) {
        int best = k + 1 < n - k ? k + 1 : n - k;
        for (int c = 0; c < n; c++) {
          int v = dy[i + (size_t)n * (j + (size_t)n * c)], e = abs(c - k);
          int m = v > e ? v : e;
          if (m < best) best = m;
        }
        if (VOX[i + (size_t)n * (j + (size_t)n * k)]) best = 0;
        DC[i + (size_t)n * (j + (size_t)n * k)] = (uint8_t)(best > capc ? capc : best);
      }
  free(dx);
  free(dy);
  for (int o = 0; o < 8; o++) {
    FO[o] = malloc(tot);
    int sx = (o & 1) ? -1 : 1, sy = (o & 2) ? -1 : 1, sz = (o & 4) ? -1 : 1;
    for (int kk = 0; kk < n; kk++) {
      int k = sz > 0 ? n - 1 - kk : kk;
      for (int jj = 0; jj < n; jj++) {
        int j = sy > 0 ? n - 1 - jj : jj;
        for (int ii = 0; ii < n; ii++) {
          int i = sx > 0 ? n - 1 - ii : ii;
          int f = 0;
          if (!occ(i, j, k)) {
            int m = 1 << 30;
            for (int q = 1; q < 8; q++) {
              int a = i + ((q & 1) ? sx : 0), b = j + ((q & 2) ? sy : 0), c = k + ((q & 4) ? sz : 0);
              int v = (a < 0 || b < 0 || c < 0 || a >= n || b >= n || c >= n)
                          ? 0 : FO[o][a + (size_t)n * (b + (size_t)n * c)];
              if (v < m) m = v;
            }
            f = m + 1;
            if (f > capo) f = capo;
          }
          FO[o][i + (size_t)n * (j + (size_t)n * k)] = (uint8_t)f;
        }
      }
    }
  }
}

static int behind_clear(int i, int j, int k, int sx, int sy, int sz) {
  for (int a = 0; a < 3; a++)
    for (int q = 0; q < 4; q++) {
      int d[3] = {0, 0, 0};
      int sv[3] = {sx, sy, sz};
      d[a] = -sv[a];
      int b = (a + 1) % 3, c = (a + 2) % 3;
      if (q & 1) d[b] = sv[b];
      if (q & 2) d[c] = sv[c];
      if (occ(i + d[0], j + d[1], k + d[2])) return 0;
    }
  return 1;
}

static inline float gmin(float a, float b) { return b < a ? b : a; }
static inline float sgn(float x) { return x > 0 ? 1.f : (x < 0 ? -1.f : 0.f); }
static inline float np1(float d, float p) { return d < 0 ? ceilf(p - 1.f) : floorf(p + 1.f); }

typedef struct {
  int steps;
  int nsamp[NS];
  /* sampled step indices (bitmap over steps, up to 4096) */
  uint64_t bm[NS][64];
  int hit;
  float hitlen;
  v3 hitpt;
} walk_t;

/* one walk; shadow: stops at opaque (byte not 0/2); primary: stops at any non-zero byte */
static void walk(v3 pos, v3 dir, float len0, float maxlen, int shadow, walk_t* w) {
  memset(w, 0, sizeof *w);
  float fn = (float)N;
  v3 st = {sgn(dir.x), sgn(dir.y), sgn(dir.z)};
  v3 t = {(np1(dir.x, pos.x) - pos.x) / dir.x, (np1(dir.y, pos.y) - pos.y) / dir.y,
          (np1(dir.z, pos.z) - pos.z) / dir.z};
  v3 rcp = {1.f / dir.x, 1.f / dir.y, 1.f / dir.z};
  int oct = (dir.x < 0 ? 1 : 0) | (dir.y < 0 ? 2 : 0) | (dir.z < 0 ? 4 : 0);
  v3 c0 = {dir.x > 0 ? 0.f : 1.f, dir.y > 0 ? 0.f : 1.f, dir.z > 0 ? 0.f : 1.f};
  float slim[NS];
  for (int s = 0; s < NS; s++) slim[s] = -1.f;
  float len = len0;
  v3 cur = pos;
  int it = 0;
  const float margin = 1.f / 256.f;
  while (len < maxlen) {
    int out = (cur.x > fn && dir.x > 0) || (cur.x < 0 && dir.x < 0) || (cur.y > fn && dir.y > 0) ||
              (cur.y < 0 && dir.y < 0) || (cur.z > fn && dir.z > 0) || (cur.z < 0 && dir.z < 0);
    if (out || it >= 4096) return;
    float tm = gmin(t.x, gmin(t.y, t.z));
    t.x -= tm; t.y -= tm; t.z -= tm;
    len += tm;
    float s = len - len0;
    cur.x = pos.x + s * dir.x; cur.y = pos.y + s * dir.y; cur.z = pos.z + s * dir.z;
    int ex = t.x == 0.f, ey = t.y == 0.f, ez = t.z == 0.f;
    v3 sp = {cur.x + 0.5f * ex * st.x, cur.y + 0.5f * ey * st.y, cur.z + 0.5f * ez * st.z};
    int inb = sp.x >= 0 && sp.y >= 0 && sp.z >= 0 && sp.x <= fn && sp.y <= fn && sp.z <= fn;
    int vi = 0, vj = 0, vk = 0;
    uint8_t b = 0;
    if (inb) {
      vi = (int)floorf(sp.x) % N; vj = (int)floorf(sp.y) % N; vk = (int)floorf(sp.z) % N;
      b = VOX[vi + (size_t)N * (vj + (size_t)N * vk)];
    }
    for (int sc = 0; sc < NS; sc++) {
      if (s < slim[sc]) continue;  /* skipped */
      w->nsamp[sc]++;
      if (it < 4096) w->bm[sc][it >> 6] |= 1ull << (it & 63);
      slim[sc] = -1.f;
      if (inb && b == 0) {
        size_t id = vi + (size_t)N * (vj + (size_t)N * vk);
        int D;
        if (sc == 0) D = DC[id];
        else if (sc == 1) D = FO[oct][id];
        else if (sc == 3 && behind_clear(vi, vj, vk, (int)st.x, (int)st.y, (int)st.z)) D = FO[oct][id];
        else {
          int a = vi - (int)st.x, bb = vj - (int)st.y, cc = vk - (int)st.z;
          D = (a < 0 || bb < 0 || cc < 0 || a >= N || bb >= N || cc >= N)
                  ? 0 : FO[oct][a + (size_t)N * (bb + (size_t)N * cc)] - 1;
          if (D < 0) D = 0;
        }
        if (D >= 2) {
          float fd = (float)D - margin;
          float lx = ((vi + c0.x) + st.x * fd - pos.x) * rcp.x;
          float ly = ((vj + c0.y) + st.y * fd - pos.y) * rcp.y;
          float lz = ((vk + c0.z) + st.z * fd - pos.z) * rcp.z;
          float l = fminf(fminf(lx, ly), fminf(lz, maxlen - len0));
          slim[sc] = l;
        }
      }
    }
    it++;
    w->steps = it;
    int ev = shadow ? (b != 0 && b != 2) : (b != 0);
    if (ev) {
      w->hit = 1;
      w->hitlen = len;
      w->hitpt = cur;
      return;
    }
    int idx = ez ? 2 : (ey ? 1 : 0);
    float pa = idx == 0 ? pos.x : (idx == 1 ? pos.y : pos.z);
    float da = idx == 0 ? dir.x : (idx == 1 ? dir.y : dir.z);
    float ca = idx == 0 ? cur.x : (idx == 1 ? cur.y : cur.z);
    float sa = idx == 0 ? st.x : (idx == 1 ? st.y : st.z);
    float q = ((ca + sa) - pa) / da - s;
    if (idx == 0) t.x = q; else if (idx == 1) t.y = q; else t.z = q;
  }
}

/* out[0..]: lane steps primary, lane steps shadow, wave steps primary, wave steps shadow,
 * then per scheme: lane samples prim, lane samples shadow, wave samples prim, wave samples shadow */
void sim_run(const float* inv_pv, int W, int H, int tile_stride, const float* sun_n, float maxlen,
             double* out) {
  int tw = W / 8, th = H / 8;
  double acc[4 + 4 * NS];
  memset(acc, 0, sizeof acc);
#pragma omp parallel
  {
    double loc[4 + 4 * NS];
    memset(loc, 0, sizeof loc);
    walk_t* wp = malloc(sizeof(walk_t) * 64);
    walk_t* ws = malloc(sizeof(walk_t) * 64);
#pragma omp for schedule(dynamic)
    for (int tile = 0; tile < tw * th; tile += tile_stride) {
      int tx = tile % tw, ty = tile / tw;
      int hasS[64];
      for (int l = 0; l < 64; l++) {
        int px = tx * 8 + (l & 7), py = ty * 8 + (l >> 3);
        float ndx = (2.f * (px + 0.5f)) / W - 1.f, ndy = (2.f * (py + 0.5f)) / H - 1.f;
        float n4[4], f4[4];
        for (int i = 0; i < 4; i++) {
          float base = inv_pv[i] * ndx + inv_pv[4 + i] * ndy;
          n4[i] = (base + inv_pv[8 + i] * -1.f) + inv_pv[12 + i];
          f4[i] = (base + inv_pv[8 + i]) + inv_pv[12 + i];
        }
        v3 nr = {n4[0] / n4[3], n4[1] / n4[3], n4[2] / n4[3]};
        v3 vd = {f4[0] / f4[3] - nr.x, f4[1] / f4[3] - nr.y, f4[2] / f4[3] - nr.z};
        float inv = 1.f / sqrtf(vd.x * vd.x + vd.y * vd.y + vd.z * vd.z);
        v3 d = {vd.x * inv, vd.y * inv, vd.z * inv};
        v3 p = {nr.x + N * 0.5f, nr.y + N * 0.5f, nr.z + N * 0.5f};
        walk(p, d, 0.f, maxlen, 0, &wp[l]);
        hasS[l] = wp[l].hit;
        if (wp[l].hit) {
          v3 sd = {sun_n[0], sun_n[1], sun_n[2]};
          walk(wp[l].hitpt, sd, wp[l].hitlen, maxlen, 1, &ws[l]);
        } else memset(&ws[l], 0, sizeof ws[l]);
      }
      int mp = 0, ms = 0;
      for (int l = 0; l < 64; l++) {
        loc[0] += wp[l].steps; loc[1] += ws[l].steps;
        if (wp[l].steps > mp) mp = wp[l].steps;
        if (ws[l].steps > ms) ms = ws[l].steps;
        for (int sc = 0; sc < NS; sc++) {
          loc[4 + 4 * sc + 0] += wp[l].nsamp[sc];
          loc[4 + 4 * sc + 1] += ws[l].nsamp[sc];
        }
      }
      loc[2] += mp; loc[3] += ms;
      for (int sc = 0; sc < NS; sc++) {
        for (int q = 0; q < 64; q++) {
          uint64_t a = 0, b = 0;
          for (int l = 0; l < 64; l++) { a |= wp[l].bm[sc][q]; b |= ws[l].bm[sc][q]; }
          loc[4 + 4 * sc + 2] += __builtin_popcountll(a);
          loc[4 + 4 * sc + 3] += __builtin_popcountll(b);
        }
      }
      (void)hasS;
    }
#pragma omp critical
    for (int i = 0; i < 4 + 4 * NS; i++) acc[i] += loc[i];
    free(wp); free(ws);
  }
  memcpy(out, acc, sizeof acc);
}
