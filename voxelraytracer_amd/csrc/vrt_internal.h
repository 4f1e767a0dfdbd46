// vrt_internal.h — the interface between the kernels (vrt_render.hip) and the C-ABI context
// (vrt_context.cpp). Not installed; include/vrt.h is the public boundary.
#ifndef VRT_INTERNAL_H
#define VRT_INTERNAL_H

#include <hip/hip_runtime.h>

#include <cstdint>

#include "vrt.h"

namespace vrt {

// Per-launch kernel arguments (by value: one kernarg segment per launch).
struct KArgs {
  float inv_pv[16];
  float rcp_w, rcp_h;  // RN(1 / width), RN(1 / height) (host IEEE division): the NDC's divisions
  float sun[3];
  float sky_sy;      // max(u_SunDir.y, 0): the skybox's sun height factor (voxel.glsl:391), uniform
  float sun_n[3];    // normalize(u_SunDir), GLSL normalize semantics (host: same IEEE ops)
  float sun_rcp[3];  // RN(1 / sun_n): the shadow walk's per-axis reciprocals (uniform)
  float time, ray_noise, refl_noise, refr_noise, max_len;
  float fn;
  int32_t n, width, height;
  int32_t row0, rows, row_step;
  int32_t row_blk_sh;  // log2 of the band's row block (ABI v11): band row i -> frame row
                       // row0 + (i >> row_blk_sh) * row_step + (i & (2^row_blk_sh - 1))
  int32_t pitch; // pixels from one band row to the next in every output/history buffer (>= width)
  uint32_t ostride;  // bytes from one direction octant's packed volume to the next (0: one volume)
  int32_t max_refl, max_transp;
  // textured mode (!_COLOR_ONLY): atlas of atlas_size^2 RGBA8 words, row 0 = bottom
  int32_t textured, atlas_size, atlas_tex_size;
  const uint32_t* atlas;
  // temporal epilogue (cur != nullptr): RGB8 store + temporal.glsl blend instead of float RGBA
  float alpha;
  const uint32_t* prev;  // last filtered frame (RGBA8 words), band-local like the output
  uint32_t* cur;         // filtered frame written here
  uint32_t* raw;         // optional: the quantised ray-trace frame (the reference's rayTrace FBO)
  // stats-free colour-only launches (vrt_set_certified): 0 exact walks only, 1 certified walks
  // for the exact path's shadow and air-medium secondary rays, 2 also whole pixels first
  int32_t cert;
  // certified bounce trees (vrt_set_cert_trees, ABI v15): colour-only certified launches settle a
  // glass primary hit's whole bounce tree by certified walks (cert_tree) where they can
  int32_t tree;
  // tile dispatch order (stats-free launches, vrt_set_tile_order): nullptr = dispatch order, else
  // the band's order buffer: three sets of kOrdClasses list counters, the per-tile wave counters,
  // two rank sets of `tiles` words and two list sets of tiles + 8 words (see ordered_tile).
  // tiles_x: tiles per row; tiles: tiles of the launch; ord_r / ord_w: the rank and list set read /
  // written; ctr_r / ctr_w / ctr_z: the counter set read / appended to / zeroed; ord_q: first-pass
  // slots per class (grid = 8 * ord_q + tiles)
  uint32_t* order;
  uint32_t tiles_x, tiles, ord_r, ord_w, ctr_r, ctr_w, ctr_z, ord_q;
  // deferred exact pass (stats-free certified launches, vrt_set_exact_pass): nullptr = the exact
  // path runs in the certified pixel's own lane; else the certified pass appends the pixels that
  // need the exact path to a list (one atomic per wave with such pixels, on one of kOrdClasses
  // segment counters by workgroup % 8) and the exact pass renders them 64 to a wave. defer: the
  // launch slot's words (2 counter sets, then the list); defer_e: the counter set of this launch
  // (the exact pass zeroes the other one for the next launch on the stream); defer_seg: list
  // words per segment (a segment holds at most ceil(tiles / 8) tiles' pixels)
  uint32_t* defer;
  uint32_t defer_e, defer_seg;
  int32_t exact_fat;  // the exact pass's short-band instance (colour-only bands of < 4 rounds of waves, lone frames)
  // adaptive exact-pass grid (VRT_EXACT_GRID_ADAPT): workgroups of this launch's exact pass (0: the
  // tiles-based default) and the slot's host-mapped word its workgroup 0 stores the batch count in
  uint32_t exact_grid;
  uint32_t* batches_out;
  // frame batches (vrt_render_temporal_batch_async, alpha 1): `nframes` frames of the same band in
  // one launch, frame f's tiles at [f * frame_tiles, (f + 1) * frame_tiles) of the grid (tiles =
  // nframes * frame_tiles); frame 0 is inv_pv / time / cur / raw above, frame f >= 1 is fb[f - 1]
  int32_t nframes;
  uint32_t frame_tiles;
  struct FrameB {
    float inv_pv[16];
    float time;
    uint32_t* cur;
    uint32_t* raw;
  } fb[7];
};
constexpr int kMaxBatch = 8;  // frames per launch (1 + the fb entries)
#if defined(VRT_EXACT_GRID_ADAPT) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_EXACT_GRID_ADAPT is an A/B knob of make variant builds"
#endif
#ifndef VRT_EXACT_GRID_ADAPT
#define VRT_EXACT_GRID_ADAPT 1
#endif

// Waves per workgroup, each rendering an 8x8 pixel tile. Two (a 16x8 tile): a finished
// workgroup frees its slots two waves at a time, so the dispatcher refills them sooner than with
// four-wave 16x16 workgroups (C3 -4.4 %, C2 -2.8 %, C4 -8.1 % per frame; one wave per workgroup:
// C3 -1.7 %, profiles/r02_s06). Images are identical at 1, 2 and 4 (A/B builds only: make variant).
#if defined(VRT_WG_WAVES) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_WG_WAVES is an A/B knob of make variant builds"
#endif
#ifndef VRT_WG_WAVES
#define VRT_WG_WAVES 2
#endif
constexpr int kWgWaves = VRT_WG_WAVES;
static_assert(kWgWaves == 1 || kWgWaves == 2 || kWgWaves == 4, "1, 2 or 4 waves per workgroup");
constexpr int kWgThreads = 64 * kWgWaves;
constexpr int kTileW = kWgWaves >= 2 ? 16 : 8;  // a workgroup's pixel tile: 16x16, 16x8 or 8x8
constexpr int kTileH = kWgWaves == 4 ? 16 : 8;
constexpr int kMaxStack = 17;               // bounce-stack entries: max_reflections + max_transparencies + 1
constexpr int kCntReplicas = 256;           // counter replicas (per-wave atomics spread over them)
constexpr uint32_t kOrdClasses = 8;         // tile-order lists: tile % 8 (the XCD of its slot)
constexpr uint32_t kOrdCtrStride = 64;      // words between list counters (one 256-byte line each)
constexpr uint32_t kOrdHdr = 3 * kOrdClasses * kOrdCtrStride;  // tile-order buffer header: 3 counter sets
#if defined(VRT_ORD_DIV) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_ORD_DIV is an A/B knob of make variant builds"
#endif
#ifndef VRT_ORD_DIV
#define VRT_ORD_DIV 4
#endif
// first-pass slots per class of a tile-order launch: tiles / (8 VRT_ORD_DIV), i.e. up to a quarter of
// the tiles in the heavy-first pass (C3: ~1600 of a part launch's 8160 tiles are heavy)
__host__ __device__ inline uint32_t ord_q_for(uint32_t tiles) {
  return (tiles + kOrdClasses * VRT_ORD_DIV - 1u) / (kOrdClasses * VRT_ORD_DIV);
}
#if defined(VRT_ORD_MIN_ROUNDS) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_ORD_MIN_ROUNDS is an A/B knob of make variant builds"
#endif
#ifndef VRT_ORD_MIN_ROUNDS  // dispatch rounds of waves from which an in-lane launch takes the tile order
#define VRT_ORD_MIN_ROUNDS 1
#endif
constexpr uint32_t kDeferHdr = 4 * kOrdClasses * kOrdCtrStride;  // deferred-pass slot header: 2 kinds x 2 sets
constexpr uint32_t kDeferDense = 32;        // deferred pixels from which a wave keeps its own exact-pass batch
#if defined(VRT_DEFER_GRID_DIV) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_DEFER_GRID_DIV is an A/B knob of make variant builds"
#endif
#ifndef VRT_DEFER_GRID_DIV
#define VRT_DEFER_GRID_DIV 8
#endif
// certified-pass waves per exact-pass workgroup (the exact pass's grid; a workgroup loops over the
// batches beyond it): 8 covers textured frames' deferred pixels in one batch per workgroup (textured
// C3 0.0843 -> 0.0713 ms against 32; 4 no better; profiles/r03_s11, r03_s12)
constexpr uint32_t kDeferGridDiv = VRT_DEFER_GRID_DIV;
#if defined(VRT_DEFER_GRID_DIV_COLOR) && !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_DEFER_GRID_DIV_COLOR is an A/B knob of make variant builds"
#endif
#ifndef VRT_DEFER_GRID_DIV_COLOR
#define VRT_DEFER_GRID_DIV_COLOR VRT_DEFER_GRID_DIV
#endif
constexpr uint32_t kDeferGridDivColor = VRT_DEFER_GRID_DIV_COLOR;  // the same for colour-only frames

// ---- launches (vrt_render.hip); all asynchronous on `s` ------------------------------------

// render_kernel: the instance is chosen from (stats, a.textured, a.cert); grid = a.tiles, or
// 8 * a.ord_q + a.tiles with a tile order (a.order). cnt_rep: the counter replicas (stats launches).
// ev_begin / ev_end (optional, timing events) are recorded when the kernel starts and ends on
// the device (hipExtLaunchKernelGGL), not when the host enqueues it.
void launch_render(const KArgs& a, bool stats, const uint16_t* vox, float4* out, vrt_hit* hit,
                   unsigned long long* cnt_rep, hipStream_t s, hipEvent_t ev_begin = nullptr,
                   hipEvent_t ev_end = nullptr);
// fold the counter replicas into dst (accumulating) and re-zero them
void launch_reduce_counters(unsigned long long* rep, unsigned long long* dst, hipStream_t s);
// the kernel's packed volume from the canonical N^3 bytes: 8 octant forward-distance volumes
// (octants == 8; tmp = 3 N^3 bytes) or one centred-distance volume (tmp = 2 N^3 bytes)
void launch_volume_passes(const uint8_t* vox, uint8_t* tmp, uint16_t* packed, uint32_t n,
                          int octants, hipStream_t s);
// glass and non-empty voxel counts into out[0..1] (accumulating)
void launch_glass_share(const uint8_t* vox, uint64_t total, unsigned long long* out, hipStream_t s);
void launch_build_scene(uint8_t* vox, int scene, uint32_t n, const float* noise, hipStream_t s);
int run_fast_math_check(unsigned long long* host_out);  // vrt_debug_fast_math (7 counters)
void launch_randomize(const float* dir, const float* pos, int n, float randomness, float seed,
                      float* out, hipStream_t s);
// frame rows [0, height) from k block-cyclic bands of 2^sh-row blocks, band_words words apart
// (band j's row i = frame row ((i >> sh) k + j) 2^sh + i % 2^sh), rows frame_pitch words apart
void launch_assemble_blocks(const uint32_t* bands, uint64_t band_words, int32_t k, int32_t sh, int32_t width,
                            int32_t height, uint32_t* frame, uint64_t frame_pitch, hipStream_t s);
// RGB8 wire format: RGBA8 words (A = 255) -> 3 bytes per pixel (pixels % 4 == 0, 16-byte aligned)
void launch_pack_rgb8(const uint32_t* rgba, uint64_t pixels, uint8_t* rgb, hipStream_t s);
// launch_assemble_blocks from RGB8 bands (band_px pixels apart), unpacked to RGBA8 words (width % 4 == 0)
void launch_assemble_blocks_rgb8(const uint8_t* bands, uint64_t band_px, int32_t k, int32_t sh, int32_t width,
                                 int32_t height, uint32_t* frame, uint64_t frame_pitch, hipStream_t s);

}  // namespace vrt

#endif  // VRT_INTERNAL_H
