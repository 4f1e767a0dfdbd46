// vrt_host.cpp — host-side scene harness of the C-ABI (no GPU needed).
//
// Mirrors the parts of src/main.cpp that produce the hot path's inputs:
//   - volume generators _TERRAIN / _GLASS_CUBE / _REFRACTION   (main.cpp:218-288)
//   - camera invPV = ~(P * V)                                    (main.cpp:67-76, 161)
//   - sun direction from the day clock                           (main.cpp:346-348)
// Greet's Noise::GenNoise, Mat4 and Vec2::Rotate are not vendored; the
// replacements are specified in DESIGN.md and are inputs to render(), not part of the parity
// contract of the kernel.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "vrt.h"

namespace {

// DESIGN.md "Terrain noise": seeded value noise replacing Greet::Noise::GenNoise(size, size,
// 5, 10, 10, persistence, 0, 0). Lattice values from a 32-bit integer mix, smoothstep-bilinear
// interpolation in double, normalised by the total amplitude, mapped to [0.2, 0.5], rounded to
// float.
uint32_t mix32(uint32_t seed, uint32_t octave, uint32_t i, uint32_t j) {
  uint32_t h = seed * 0x9E3779B1u ^ octave * 0x85EBCA77u ^ i * 0xC2B2AE3Du ^ j * 0x27D4EB2Fu;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

double lattice_value(uint32_t seed, int octave, int i, int j) {
  const uint32_t h = mix32(seed, uint32_t(octave), uint32_t(i), uint32_t(j));
  return double(h >> 8) * (1.0 / 16777216.0);
}

double smooth(double f) { return f * f * (3.0 - 2.0 * f); }

struct Mat4d {
  double m[16] = {0};  // column-major m[col*4 + row], as GL
  static Mat4d identity() {
    Mat4d r;
    r.m[0] = r.m[5] = r.m[10] = r.m[15] = 1.0;
    return r;
  }
  double& at(int row, int col) { return m[col * 4 + row]; }
  double at(int row, int col) const { return m[col * 4 + row]; }
  Mat4d operator*(const Mat4d& b) const {
    Mat4d r;
    for (int row = 0; row < 4; ++row)
      for (int col = 0; col < 4; ++col) {
        double s = 0.0;
        for (int k = 0; k < 4; ++k) s += at(row, k) * b.at(k, col);
        r.at(row, col) = s;
      }
    return r;
  }
};

Mat4d perspective(double aspect, double fov_deg, double n, double f) {
  const double t = 1.0 / std::tan(fov_deg * M_PI / 360.0);
  Mat4d p;
  p.at(0, 0) = t / aspect;
  p.at(1, 1) = t;
  p.at(2, 2) = (f + n) / (n - f);
  p.at(2, 3) = 2.0 * f * n / (n - f);
  p.at(3, 2) = -1.0;
  return p;
}

Mat4d rotate_x(double deg) {
  const double r = deg * M_PI / 180.0, c = std::cos(r), s = std::sin(r);
  Mat4d m = Mat4d::identity();
  m.at(1, 1) = c;
  m.at(1, 2) = -s;
  m.at(2, 1) = s;
  m.at(2, 2) = c;
  return m;
}

Mat4d rotate_y(double deg) {
  const double r = deg * M_PI / 180.0, c = std::cos(r), s = std::sin(r);
  Mat4d m = Mat4d::identity();
  m.at(0, 0) = c;
  m.at(0, 2) = s;
  m.at(2, 0) = -s;
  m.at(2, 2) = c;
  return m;
}

Mat4d translate(double x, double y, double z) {
  Mat4d m = Mat4d::identity();
  m.at(0, 3) = x;
  m.at(1, 3) = y;
  m.at(2, 3) = z;
  return m;
}

// Gauss-Jordan inverse with partial pivoting; false if singular.
bool invert(const Mat4d& a, Mat4d* out) {
  double w[4][8];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 8; ++c) w[r][c] = c < 4 ? a.at(r, c) : (c - 4 == r ? 1.0 : 0.0);
  for (int c = 0; c < 4; ++c) {
    int piv = c;
    for (int r = c + 1; r < 4; ++r)
      if (std::fabs(w[r][c]) > std::fabs(w[piv][c])) piv = r;
    if (std::fabs(w[piv][c]) < 1e-300) return false;
    if (piv != c)
      for (int k = 0; k < 8; ++k) std::swap(w[c][k], w[piv][k]);
    const double inv = 1.0 / w[c][c];
    for (int k = 0; k < 8; ++k) w[c][k] *= inv;
    for (int r = 0; r < 4; ++r) {
      if (r == c) continue;
      const double f = w[r][c];
      for (int k = 0; k < 8; ++k) w[r][k] -= f * w[c][k];
    }
  }
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) out->at(r, c) = w[r][c + 4];
  return true;
}

}  // namespace

extern "C" {

int vrt_abi_version(void) { return VRT_ABI_VERSION; }

int vrt_terrain_noise(int32_t n, uint32_t seed, float* out) {
  if (n <= 0 || !out) return VRT_ERR_INVALID;
  const int octaves = 5;
  const double persistence = n <= 32 ? 0.5 : 0.125;  // main.cpp:185 (_HIGH_PERFORMANCE) / :195
  for (int z = 0; z < n; ++z) {
    for (int x = 0; x < n; ++x) {
      double sum = 0.0, total = 0.0, amp = 1.0;
      for (int o = 0; o < octaves; ++o) {
        const int step = std::max(1, n / (4 << o));  // lattice spacing: n/4, n/8, ...
        const int i0 = x / step, j0 = z / step;
        const double fx = smooth(double(x - i0 * step) / double(step));
        const double fz = smooth(double(z - j0 * step) / double(step));
        const double a = lattice_value(seed, o, i0, j0);
        const double b = lattice_value(seed, o, i0 + 1, j0);
        const double c = lattice_value(seed, o, i0, j0 + 1);
        const double d = lattice_value(seed, o, i0 + 1, j0 + 1);
        const double top = a + (b - a) * fx;
        const double bot = c + (d - c) * fx;
        sum += amp * (top + (bot - top) * fz);
        total += amp;
        amp *= persistence;
      }
      // rolling hills between 0.2 N and 0.5 N: the default camera (main.cpp:171) stays above them
      float v = float(0.2 + 0.3 * (sum / total));
      if (v >= 1.0f) v = 0x1.fffffep-1f;
      if (v < 0.0f) v = 0.0f;
      out[x + z * n] = v;
    }
  }
  return VRT_OK;
}

int vrt_build_scene(int32_t scene, int32_t n, uint32_t seed, uint8_t* data) {
  if (!data || n < 8 || n > 1024) return VRT_ERR_INVALID;
  const unsigned size = unsigned(n);
  const size_t plane = size_t(size) * size;
  std::memset(data, 0, plane * size);
  auto at = [&](size_t x, size_t y, size_t z) -> uint8_t& { return data[x + y * size + z * plane]; };
  switch (scene) {
    case VRT_SCENE_TERRAIN: {  // main.cpp:219-257
      std::vector<float> noise(plane);
      vrt_terrain_noise(n, seed, noise.data());
      const float fs = float(size);
      for (unsigned z = 0; z < size; ++z)
        for (unsigned x = 0; x < size; ++x) {
          const float h = noise[x + z * size] * fs;
          for (int y = 0; float(y) < h; ++y) at(x, y, z) = 1;  // stone
          at(x, size_t(int(h)), z) = 3;                         // grass cap
        }
      if (size <= 64) {  // glass walls only on small volumes (main.cpp:233)
        for (unsigned z = 2; z < size - 2; ++z)
          for (int y = int(noise[z * size] * fs + 1.0f); y < int(size); ++y) at(0, y, z) = 2;
        for (unsigned x = 2; x < size - 1; ++x)
          for (int y = int(noise[x * size + size - 4] * fs + 1.0f); y < int(size) - 4; ++y)
            at(x, y, size - 4) = 2;
      }
      for (unsigned z = 2; z < size - 2; ++z)
        for (int y = int(noise[size - 1 + z * size] * fs + 1.0f); y < int(size) - 4; ++y)
          at(size - 1, y, z) = 3;
      break;
    }
    case VRT_SCENE_GLASS_CUBE:  // main.cpp:258-271: six glass faces, grass voxel in the centre
      for (size_t i = 0; i < size; ++i)
        for (size_t j = 0; j < size; ++j) {
          at(size - 1, i, j) = 2;
          at(0, i, j) = 2;
          at(i, j, size - 1) = 2;
          at(i, j, 0) = 2;
          at(i, size - 1, j) = 2;
          at(i, 0, j) = 2;
        }
      at(size / 2, size / 2, size / 2) = 3;
      break;
    case VRT_SCENE_REFRACTION:  // main.cpp:272-287: glass voxel in the centre, grass panels
      at(size / 2, size / 2, size / 2) = 2;
      for (size_t i = size / 4; i < 3 * size / 4; ++i)
        for (size_t j = size / 4; j < 3 * size / 4; ++j) {
          at(size - 1, i, j) = 3;
          at(0, i, j) = 3;
          at(i, j, size - 1) = 3;
          at(i, j, 0) = 3;
          at(i, size - 1, j) = 3;
          at(i, 0, j) = 3;
        }
      break;
    default:
      return VRT_ERR_INVALID;
  }
  return VRT_OK;
}

int vrt_camera_make(const float pos[3], const float rot_deg[3], int32_t width, int32_t height,
                    float fov_deg, float near_plane, float far_plane, vrt_camera* out) {
  if (!pos || !rot_deg || !out || width <= 0 || height <= 0) return VRT_ERR_INVALID;
  const Mat4d p = perspective(double(width) / double(height), fov_deg, near_plane, far_plane);
  const Mat4d v = rotate_x(-double(rot_deg[0])) * rotate_y(-double(rot_deg[1])) *
                  translate(-double(pos[0]), -double(pos[1]), -double(pos[2]));
  Mat4d inv;
  if (!invert(p * v, &inv)) return VRT_ERR_INVALID;
  for (int i = 0; i < 16; ++i) out->inv_pv[i] = float(inv.m[i]);
  out->width = width;
  out->height = height;
  return VRT_OK;
}

void vrt_sun_dir(float time_of_day, float day_time, float out[3]) {
  // Vec2f dir{1,0}; dir.Rotate(timeOfDay*pi*2/dayTime); u_SunDir = normalize(dir.y, dir.x, 0.2)
  const double a = double(time_of_day) * M_PI * 2.0 / double(day_time);
  const float dx = float(std::cos(a)), dy = float(std::sin(a));
  const float l = std::sqrt(dy * dy + dx * dx + 0.2f * 0.2f);
  out[0] = dy / l;
  out[1] = dx / l;
  out[2] = 0.2f / l;
}

void vrt_params_default(vrt_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  vrt_sun_dir(0.9f * 50.0f, 50.0f, p->sun_dir);  // "Make day" (main.cpp:577)
  p->time = 1.0f;
  p->max_ray_length = 100.0f;
  p->max_reflections = 1;
  p->max_transparencies = 2;
  p->color_only = 1;
}

}  // extern "C"
