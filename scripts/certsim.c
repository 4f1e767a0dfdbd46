/* Certified-walk simulator (analysis tool; not product, not oracle). Replays the primary and
 * shadow walks of the reference exactly (the oracle's march / march_shadow, voxel.glsl:259-384)
 * and, beside them, a CERTIFIED walk: a float DDA over the real ray with empty-space jumps that
 * returns the exact walk's outcome (primary: first event byte + face axis; shadow: blocked or not)
 * only when no float rounding of the exact walk can change it, and UNCERTAIN otherwise.
 * Counts iterations, uncertain rays (per lane and per 8x8 wave) and any disagreement.
 * Build/run: python scripts/certsim.py --config C3
 */
#include "../oracle/vrt_oracle.c"

#include <stdio.h>

static int N;
static const uint8_t* VOX;
static uint8_t* FO[8];
static double GSCALE = 1.0;   /* experiment: scale the rounding bounds (1 = the derived bound) */
static float MARGIN = 1.0f / 64.0f;

static inline int occ(int i, int j, int k) {
  if (i < 0 || j < 0 || k < 0 || i >= N || j >= N || k >= N) return 1;
  return VOX[i + (size_t)N * (j + (size_t)N * k)] != 0;
}

EXPORT void cs_build(const uint8_t* vox, int n, int cap) {
  N = n;
  VOX = vox;
  size_t tot = (size_t)n * n * n;
  for (int o = 0; o < 8; o++) {
    free(FO[o]);
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
            if (f > cap) f = cap;
          }
          FO[o][i + (size_t)n * (j + (size_t)n * k)] = (uint8_t)f;
        }
      }
    }
  }
}

/* byte on the certified path: cells with an index outside [0, N) are outside (0) — the exact walk
 * reads plane N (GL_REPEAT) only at a coordinate exactly N, i.e. at a near-edge crossing */
static inline int path_byte(const int c[3]) {
  if (c[0] < 0 || c[1] < 0 || c[2] < 0 || c[0] >= N || c[1] >= N || c[2] >= N) return 0;
  return VOX[c[0] + (size_t)N * (c[1] + (size_t)N * c[2])];
}
/* byte of an alternative cell (near-edge): index N may be the wrapped plane 0 */
static inline int alt_byte(const int c[3]) {
  int i = c[0], j = c[1], k = c[2];
  if (i < 0 || j < 0 || k < 0 || i > N || j > N || k > N) return 0;
  if (i == N) i = 0;
  if (j == N) j = 0;
  if (k == N) k = 0;
  return VOX[i + (size_t)N * (j + (size_t)N * k)];
}
static inline int is_event(int b, int shadow) { return shadow ? (b != 0 && b != 2) : (b != 0); }

/* G(v) = F(v - s) - 1: the box [v - s, v + (G - 1) s] is empty and in the volume */
static inline int gdist(const int c[3], const int s[3], int o) {
  int u[3] = {c[0] - s[0], c[1] - s[1], c[2] - s[2]};
  for (int a = 0; a < 3; a++) {
    if (c[a] < 0 || c[a] >= N || u[a] < 0 || u[a] >= N) return 0;
  }
  return (int)FO[o][u[0] + (size_t)N * (u[1] + (size_t)N * u[2])] - 1;
}

enum { C_MISS = 0, C_HIT = 1, C_UNC = 2 };
typedef struct {
  int res, byte, axis, cell[3];
  float u;      /* crossing parameter of the hit */
  float eu;     /* bound of the exact walk's parameter error there */
  int iters, jumps;
  int why;      /* reason of UNC */
} cres_t;

static const double U24 = 1.0 / 16777216.0;

/* Certified walk from P along D (all |d| normal), budget U = max_len - len0 (the exact walk
 * samples the crossing at u iff its len before that step < max_len). cell0: start cell (NULL:
 * the exact walk's own start convention). e0: extra parameter uncertainty at the start (shadow
 * origin), ed[3]: extra per-axis crossing-order uncertainty (shadow origin). */
static cres_t cwalk(v3 P, v3 D, float U, int shadow, const int* cell0, double e0,
                    const double ed[3], double len0b) {
  cres_t r;
  memset(&r, 0, sizeof r);
  float p[3] = {P.x, P.y, P.z}, d[3] = {D.x, D.y, D.z};
  for (int a = 0; a < 3; a++)   /* the kernel's fast_path_ok: the exact walk handles the rest */
    if (!(fabsf(d[a]) >= 0x1p-64f && fabsf(d[a]) <= 1.0e4f)) { r.res = C_UNC; r.why = 1; return r; }
  int s[3], cell[3];
  float rcp[3], arcp[3], sig[3];
  double l1 = 0.0;
  int o = 0;
  for (int a = 0; a < 3; a++) {
    s[a] = d[a] > 0.0f ? 1 : -1;
    rcp[a] = 1.0f / d[a];
    arcp[a] = fabsf(rcp[a]);
    l1 += fabs(d[a]);
    if (d[a] < 0.0f) o |= 1 << a;
    cell[a] = cell0 ? cell0[a] : (d[a] > 0.0f ? (int)floorf(p[a]) : (int)ceilf(p[a]) - 1);
    float np = (float)(cell[a] + (s[a] > 0 ? 1 : 0));
    sig[a] = (np - p[a]) * rcp[a];
  }
  for (int a = 0; a < 3; a++)
    if (cell[a] < 0 || cell[a] >= N) { r.res = C_UNC; r.why = 1; return r; }
  int first = 1;
  for (int guard = 0; guard < 100000; guard++) {
    r.iters++;
    int a = 0;
    if (sig[1] < sig[a]) a = 1;
    if (sig[2] < sig[a]) a = 2;
    const float s1 = sig[a];
    /* rounding bounds at this parameter: K exact-walk steps so far */
    /* non-zero exact-walk steps up to u: at most u*|d|_1 + 3 (zero-length tie steps add no
     * rounding); len_k <= (k + 3)/|d|_1 + len0, so the len additions err by at most
     * 2^-24 * sum_k len_k; each crossing's t is re-anchored from currentPos (3 roundings of
     * magnitude <= N + 2, scaled by 1/|d_b|) and then decremented at most K times */
    const double uu = (s1 > 0 ? s1 : 0);
    const double K = uu * l1 + 3.0;
    const double sumlen = (K + 3.0) * (K + 3.0) / (2.0 * l1) + K * (len0b + 1.0);
    double gam[3];
    for (int b = 0; b < 3; b++)
      gam[b] = GSCALE * (U24 * (sumlen + (K + 3.0 * N + 8.0) * arcp[b] + 2.0 * (uu + len0b)) +
                         4e-5 + e0 + ed[b]);
    const double gL = GSCALE * (2.0 * U24 * sumlen + 1e-4 + e0);
    /* empty-space jump */
    int G = gdist(cell, s, o);
    if (first) {   /* no crossing behind the start: the unguarded box F(v) = G(v + s) + 1 */
      int c2[3] = {cell[0] + s[0], cell[1] + s[1], cell[2] + s[2]};
      G = gdist(c2, s, o) + 1;
      first = 0;
    }
    if (G >= 2) {
      /* per axis: box face of axis b minus that axis's crossing bound (the kernel's rule) */
      float uj = U + 2.0f;
      for (int b = 0; b < 3; b++) {
        float face = (float)(s[b] > 0 ? cell[b] + G : cell[b] + 1 - G) - (float)s[b] * MARGIN;
        float l = (face - p[b]) * rcp[b];
        float lb = (float)(l - gam[b]);
        if (lb < uj) uj = lb;
      }
      if (uj > s1) {
        for (int b = 0; b < 3; b++) {
          float x = p[b] + uj * d[b];
          cell[b] = s[b] > 0 ? (int)floorf(x) : (int)ceilf(x) - 1;
          float np = (float)(cell[b] + (s[b] > 0 ? 1 : 0));
          sig[b] = (np - p[b]) * rcp[b];
        }
        r.jumps++;
        continue;
      }
    }
    /* one crossing: s1 on axis a */
    float prev = 0.0f;
    for (int b = 0; b < 3; b++) {
      float q = sig[b] - arcp[b];
      if (q > prev) prev = q;
    }
    if ((double)prev > (double)U + gL) { r.res = C_MISS; return r; }
    int nc[3] = {cell[0], cell[1], cell[2]};
    nc[a] += s[a];
    int nah = 0, nbh = 0, ah[3] = {0, 0, 0}, bh[3] = {0, 0, 0};
    for (int b = 0; b < 3; b++) {
      if (b == a) continue;
      if ((double)sig[b] - s1 < gam[a] + gam[b]) { ah[b] = 1; nah++; }
      float q = sig[b] - arcp[b];
      if (q >= 0.0f && (double)s1 - q < gam[a] + gam[b]) { bh[b] = 1; nbh++; }
    }
    const int ev = is_event(path_byte(nc), shadow);
    if (ev) {
      if (shadow && (nah || nbh) && nah + nbh < 2) {
        /* blocked whichever order the exact walk takes: near-behind b still samples nc (or
         * nc - e_b first); near-ahead b samples nc, or cell + e_b and then nc + e_b */
        int ok = 1;
        for (int b = 0; b < 3; b++) {
          if (!ah[b]) continue;
          int c1[3] = {cell[0], cell[1], cell[2]}, c2[3] = {nc[0], nc[1], nc[2]};
          c1[b] += s[b];
          c2[b] += s[b];
          if (!is_event(alt_byte(c1), 1) && !is_event(alt_byte(c2), 1)) ok = 0;
        }
        if (ok && (double)prev + gL < (double)U) { r.res = C_HIT; r.byte = path_byte(nc); r.axis = a; return r; }
      }
      if (nah || nbh) { r.res = C_UNC; r.why = 2; return r; }
      if ((double)prev + gL >= (double)U) { r.res = C_UNC; r.why = 3; return r; }
      r.res = C_HIT;
      r.byte = path_byte(nc);
      r.axis = a;
      memcpy(r.cell, nc, sizeof nc);
      r.u = s1;
      r.eu = gam[a];
      return r;
    }
    if (nah + nbh >= 2) {   /* near a corner: every cell of the 2x2x2 block ahead */
      for (int q = 1; q < 8; q++) {
        int c[3] = {cell[0] + ((q & 1) ? s[0] : 0), cell[1] + ((q & 2) ? s[1] : 0),
                    cell[2] + ((q & 4) ? s[2] : 0)};
        if (is_event(alt_byte(c), shadow)) { r.res = C_UNC; r.why = 4; return r; }
      }
      for (int b = 0; b < 3; b++) {
        if (!bh[b]) continue;
        int c[3] = {nc[0], nc[1], nc[2]};
        c[b] -= s[b];
        if (is_event(alt_byte(c), shadow)) { r.res = C_UNC; r.why = 4; return r; }
      }
    } else {
      for (int b = 0; b < 3; b++) {
        if (ah[b]) {   /* b may be crossed first (or tie): cell + e_b; the tie cell is the path's */
          int c[3] = {cell[0], cell[1], cell[2]};
          c[b] += s[b];
          if (is_event(alt_byte(c), shadow)) { r.res = C_UNC; r.why = 5; return r; }
          int c2[3] = {nc[0], nc[1], nc[2]};
          c2[b] += s[b];
          if (is_event(alt_byte(c2), shadow)) { r.res = C_UNC; r.why = 5; return r; }
        }
        if (bh[b]) {   /* a may have been crossed before b: nc - e_b */
          int c[3] = {nc[0], nc[1], nc[2]};
          c[b] -= s[b];
          if (is_event(alt_byte(c), shadow)) { r.res = C_UNC; r.why = 6; return r; }
        }
      }
    }
    /* the alternatives through a wrapped plane N are covered by alt_byte */
    if ((s[a] > 0 && nc[a] >= N) || (s[a] < 0 && nc[a] < 0)) { r.res = C_MISS; return r; }
    cell[a] = nc[a];
    float np = (float)(cell[a] + (s[a] > 0 ? 1 : 0));
    sig[a] = (np - p[a]) * rcp[a];
  }
  r.res = C_UNC;
  r.why = 7;
  return r;
}

/* stats: see cs_run */
EXPORT void cs_run(const float* inv_pv, int w, int h, const float* sun, float max_len,
                   double gscale, float margin, double* out) {
  GSCALE = gscale;
  MARGIN = margin;
  ctx_t c;
  memset(&c, 0, sizeof c);
  c.vox = VOX;
  c.n = N;
  c.fn = (float)N;
  c.sun = mk(sun[0], sun[1], sun[2]);
  c.max_len = max_len;
  c.inv_pv = inv_pv;
  c.width = w;
  c.height = h;
  const int tw = (w + 7) / 8, th = (h + 7) / 8;
  double acc[32] = {0};
  uint8_t* wave_unc = calloc((size_t)tw * th, 1);
  uint16_t* wave_it = calloc((size_t)tw * th, 2);
  uint16_t* wave_its = calloc((size_t)tw * th, 2);
  uint8_t* wave_unc_p = calloc((size_t)tw * th, 1);
#pragma omp parallel
  {
    double loc[32] = {0};
#pragma omp for schedule(dynamic, 4)
    for (int py = 0; py < h; py++) {
      for (int px = 0; px < w; px++) {
        float ndx = (2.0f * ((float)px + 0.5f)) / (float)w - 1.0f;
        float ndy = (2.0f * ((float)py + 0.5f)) / (float)h - 1.0f;
        const float* m = inv_pv;
        float n4[4], f4[4];
        for (int i = 0; i < 4; i++) {
          n4[i] = ((m[0 * 4 + i] * ndx + m[1 * 4 + i] * ndy) + m[2 * 4 + i] * -1.0f) + m[3 * 4 + i] * 1.0f;
          f4[i] = ((m[0 * 4 + i] * ndx + m[1 * 4 + i] * ndy) + m[2 * 4 + i] * 1.0f) + m[3 * 4 + i] * 1.0f;
        }
        v3 vnear = mk(n4[0] / n4[3], n4[1] / n4[3], n4[2] / n4[3]);
        v3 vdir = sub(mk(f4[0] / f4[3], f4[1] / f4[3], f4[2] / f4[3]), vnear);
        ray_t ray;
        ray.pos = adds(vnear, c.fn * 0.5f);
        ray.dir = randomize_direction(normalize(vdir), vnear, 0.0f, 1.0f);
        ray.len = 0.0f;
        ray.energy = 1.0f;
        ray.voxel = 0;
        ray.rdepth = ray.tdepth = 0;
        cnt_t k;
        uint32_t steps = 0, flags = 0;
        memset(&k, 0, sizeof k);
        ray_t r0 = ray;
        isect_t is = march(&c, &r0, &k, &steps, &flags);
        loc[0] += 1;
        loc[1] += steps;
        int unc = 0, uncp = 0;
        cres_t cr = cwalk(ray.pos, ray.dir, max_len - 0.0f, 0, NULL, 0.0, (double[3]){0, 0, 0}, 0.0);
        loc[2] += cr.iters;
        { uint16_t* w = &wave_it[(py / 8) * tw + px / 8]; if (cr.iters > *w) *w = (uint16_t)cr.iters; }
        loc[3] += cr.jumps;
        if (cr.res == C_UNC) { loc[4] += 1; unc = uncp = 1; loc[20 + (cr.why & 7)] += 1; }
        else if (cr.res == C_MISS) {
          loc[5] += 1;
          if (is.found) { loc[6] += 1; if (loc[6] < 5) fprintf(stderr, "MISMATCH miss px %d %d\n", px, py); }
        } else {
          loc[7] += 1;
          if (!is.found || is.voxel != cr.byte || is.index != cr.axis) {
            loc[6] += 1;
            if (loc[6] < 5)
              fprintf(stderr, "MISMATCH hit px %d %d exact found %d byte %d idx %d  cert byte %d axis %d\n",
                      px, py, is.found, is.found ? is.voxel : -1, is.index, cr.byte, cr.axis);
          }
        }
        /* shadow of the exact hit (only meaningful where the primary is non-glass) */
        if (is.found && is.voxel != 2) {
          ray_t sr;
          sr.voxel = is.voxel;
          sr.pos = is.point;
          sr.dir = normalize(c.sun);
          sr.len = is.len;
          sr.energy = 1.0f;
          sr.rdepth = sr.tdepth = 0;
          uint32_t st2 = 0;
          int ins = march_shadow(&c, &sr, &k, &st2, &flags);
          loc[8] += 1;
          loc[9] += st2;
          const material_t* mt = material(&c, is.voxel);
          float nd = dot(is.normal, sr.dir);
          float diffuse = mt->diffuse * gmax(nd, 0.0f);
          float spec = mt->specularity * gpow(gmax(dot(reflect(sr.dir, is.normal), ray.dir), 0.0f), mt->exponent);
          if (diffuse + spec == 0.0f) {
            loc[10] += 1;   /* shadow irrelevant: lit brightness == ambient */
          } else if (cr.res != C_HIT) {
            loc[11] += 1;   /* primary not certified: shadow falls back with it */
          } else if (!(nd > 0.0f)) {
            loc[12] += 1; unc = 1;  /* back face with specular: uncertain */
          } else {
            /* certified primary hit: shadow from the certified hit point */
            int ax = cr.axis;
            float xu = cr.u;
            v3 X = add(ray.pos, sclf(xu, ray.dir));
            int c0[3] = {cr.cell[0], cr.cell[1], cr.cell[2]};
            /* the air-side cell: one back along the primary's step on the face axis */
            c0[ax] -= ray.dir.x * (ax == 0) + ray.dir.y * (ax == 1) + ray.dir.z * (ax == 2) > 0 ? 1 : -1;
            double eH = cr.eu;   /* primary parameter error at the hit */
            float Sd[3] = {sr.dir.x, sr.dir.y, sr.dir.z}, Dd[3] = {ray.dir.x, ray.dir.y, ray.dir.z};
            double ed[3];
            for (int b = 0; b < 3; b++) ed[b] = eH * fabs(Dd[b]) / fabs(Sd[b]) * 2.0;
            /* start: the origin may lie inside H by eH*|D_a|; no other crossing may come first */
            int okst = 1;
            float Xa[3] = {X.x, X.y, X.z};
            for (int b = 0; b < 3; b++) {
              if (b == ax) continue;
              float np = (float)(c0[b] + (Sd[b] > 0 ? 1 : 0));
              float wb = (np - Xa[b]) / Sd[b];
              if (wb < (eH * fabs(Dd[ax]) + 1e-5) / fabs(Sd[ax]) + ed[b] + 1e-4) okst = 0;
            }
            if (!okst) { loc[13] += 1; unc = 1; }
            else {
              cres_t cs = cwalk(X, sr.dir, max_len - is.len, 1, c0, eH, ed, xu);
              loc[14] += cs.iters;
              { uint16_t* w = &wave_its[(py / 8) * tw + px / 8]; if (cs.iters > *w) *w = (uint16_t)cs.iters; }
              loc[15] += cs.jumps;
              if (cs.res == C_UNC) { loc[16] += 1; unc = 1; loc[24 + (cs.why & 7)] += 1; }
              else {
                loc[17] += 1;
                if ((cs.res == C_HIT) != (ins != 0)) {
                  loc[18] += 1;
                  if (loc[18] < 5) fprintf(stderr, "MISMATCH shadow px %d %d exact %d cert %d\n", px, py, ins, cs.res);
                }
              }
            }
          }
        }
        if (unc) wave_unc[(py / 8) * tw + px / 8] = 1;
        if (uncp) wave_unc_p[(py / 8) * tw + px / 8] = 1;
        loc[19] += unc;
      }
    }
#pragma omp critical
    for (int q = 0; q < 32; q++) acc[q] += loc[q];
  }
  double wu = 0, wup = 0;
  double wi = 0, wis = 0;
  for (int i = 0; i < tw * th; i++) { wu += wave_unc[i]; wup += wave_unc_p[i]; wi += wave_it[i]; wis += wave_its[i]; }
  fprintf(stderr, "wave-level iterations (max over 8x8): primary %.2f shadow %.2f per wave\n", wi / (tw * th), wis / (tw * th));
  free(wave_it);
  free(wave_its);
  free(wave_unc);
  free(wave_unc_p);
  for (int q = 0; q < 32; q++) out[q] = acc[q];
  out[30] = wu / (tw * th);
  out[31] = wup / (tw * th);
}
