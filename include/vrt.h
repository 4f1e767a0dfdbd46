/*
 * vrt.h — C-ABI drop-in boundary of the MI355X-native voxel ray tracer.
 *
 * Replaces the reference's GL boundary for the per-pixel ray-trace pass:
 *   - 3D-texture upload      src/main.cpp:315-319  (glTexImage3D GL_RED/UNSIGNED_BYTE, NEAREST)
 *   - uniforms + quad draw    src/main.cpp:325-361  (u_PVInvMatrix, u_Size, u_SunDir, u_Time, noises)
 *   - RGB colour FBO          src/FrameBuffer.cpp:5-19
 * and executes the program in res/shaders/voxel.glsl (fragment :1-452, vertex :454-475)
 * as a hand-written gfx950 HIP kernel.
 *
 * Conventions
 *   - Plain C types only; no exceptions cross the ABI; every entry point returns a vrt_status
 *     (0 = ok, <0 = error) and sets a per-context message readable with vrt_last_error().
 *   - Not thread-safe per context: one context per host thread (as the GL context was).
 *   - Volumes are N^3 bytes, x fastest: idx = x + y*N + z*N*N   (main.cpp:227).
 *   - Images are W*H RGBA float, row 0 = bottom row (GL window convention).
 *   - A context spans one or more GPUs (vrt_create's device mask). Whole-frame entry points
 *     (vrt_render, vrt_render_frame, vrt_render_frame_device) split the frame over k > 1 devices
 *     into block-cyclic bands of 16 adjacent rows (ABI v12; device j renders row blocks j, j+k,
 *     ..., one launch per band; vrt_frame_row_block), rendered on context-owned streams: frame f
 *     on lane f % 4. On one device a frame that runs alone (synchronous calls) or reads its
 *     history is two interleaved row parts on two streams (a synchronous colour-only certified
 *     frame of a glass-heavy volume or of >= 8 rounds of resident waves: one deferred launch, see
 *     vrt_set_exact_pass); a device-output frame at u_Alpha = 1
 *     is one launch, and up to four frames are in flight (ABI v9). The *_async band entry points
 *     run on the context's first (root) device.
 */
#ifndef VRT_H
#define VRT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VRT_ABI_VERSION 15

typedef struct vrt_ctx vrt_ctx;

typedef enum {
  VRT_OK = 0,
  VRT_ERR_INVALID = -1,      /* bad argument (null pointer, size, unsupported N) */
  VRT_ERR_DEVICE = -2,       /* HIP runtime error (message has the hipError string) */
  VRT_ERR_NO_VOLUME = -3,    /* vrt_render before vrt_upload_volume */
  VRT_ERR_OOM = -4,          /* device allocation failed */
  VRT_ERR_UNSUPPORTED = -5   /* parameter combination not built (see vrt_last_error) */
} vrt_status;

/* Camera: u_PVInvMatrix (voxel.glsl:464, set at main.cpp:333) plus the FBO size. */
typedef struct {
  float inv_pv[16];   /* column-major, GL convention: m[col*4 + row] */
  int32_t width;
  int32_t height;
} vrt_camera;

/* Volume: the bytes main.cpp:218-288 builds and :318 uploads. */
typedef struct {
  const uint8_t* voxels; /* host pointer, N^3 bytes, x fastest */
  int32_t n;             /* u_Size (voxel.glsl:18) */
} vrt_volume;

/* Per-frame parameters: the remaining uniforms (main.cpp:335-348) and compile-time switches. */
typedef struct {
  float sun_dir[3];           /* u_SunDir (main.cpp:346-348); the shader re-normalises it */
  float time;                 /* u_Time, the frame counter as float (main.cpp:343-345) */
  float ray_noise;            /* u_RayNoise        [0, 0.05] */
  float reflection_noise;     /* u_ReflectionNoise [0, 0.05] */
  float refraction_noise;     /* u_RefractionNoise [0, 0.01] */
  float max_ray_length;       /* u_MaxRayLength, default 100 (voxel.glsl:17) */
  int32_t max_reflections;    /* MAX_REFLECTIONS   (voxel.glsl:4), 0..8 */
  int32_t max_transparencies; /* MAX_TRANSPARENCIES (voxel.glsl:5), 0..8 */
  int32_t color_only;         /* _COLOR_ONLY (voxel.glsl:6): 1 colour-only, 0 textured */
  int32_t reserved0;
  const uint8_t* atlas_rgba;  /* textured mode: u_TextureUnit atlas (see vrt_upload_atlas) */
  int32_t atlas_size;         /* u_AtlasSize */
  int32_t atlas_texture_size; /* u_AtlasTextureSize */
} vrt_params;

/* Per-pixel record of the PRIMARY ray (the first stack pop, voxel.glsl:430-437). Parity key:
 * bit-exact between the HIP kernel and the CPU oracle. */
typedef struct {
  int32_t voxel_index;  /* linear index of the hit voxel (the texel GetVoxel read), -1 = no hit */
  float ray_length;     /* RayIntersection.rayLength of the primary hit (0 if none) */
  uint32_t steps;       /* DDA + shadow-DDA iterations spent on the whole pixel */
  uint32_t flags;       /* VRT_HIT_FLAG_* */
} vrt_hit;

#define VRT_HIT_FLAG_TIE3 1u        /* a y+z (or x+y+z) zero-t tie read intersectionAxis[3] (clamped to 2) */
#define VRT_HIT_FLAG_STEP_CAP 2u    /* a march hit VRT_MAX_STEPS (the GLSL would spin) */
#define VRT_HIT_FLAG_STACK_FULL 4u  /* a push was dropped (cannot happen for stack = R+T+1) */

#define VRT_MAX_STEPS 4096          /* per RayMarch / RayMarchShadow call */

/* Counter slots (uint64 each) accumulated by a render. Algorithmic bytes of a frame:
 *   DDA_STEPS + SHADOW_STEPS + 2*REFRACTION_PROBES + 16*PIXELS */
enum {
  VRT_CNT_PIXELS = 0,
  VRT_CNT_PRIMARY_RAYS,
  VRT_CNT_SECONDARY_RAYS,     /* stack pops after the primary */
  VRT_CNT_SHADOW_RAYS,        /* RayMarchShadow calls */
  VRT_CNT_DDA_STEPS,          /* RayMarch iterations that called GetVoxel */
  VRT_CNT_SHADOW_STEPS,       /* RayMarchShadow iterations that called GetVoxel */
  VRT_CNT_REFRACTION_PROBES,  /* GetRefractionRay calls (2 voxel reads each) */
  VRT_CNT_TIE3,               /* index==3 tie events */
  VRT_CNT_STEP_CAP,           /* marches cut by VRT_MAX_STEPS */
  VRT_CNT_COUNT
};

/* Statistics of a synchronous render. kernel_ms is always filled: the GPU time of the frame's
 * launches (hipEvents, the max over the context's devices), like the reference's GL_TIME_ELAPSED
 * query (main.cpp:350-360). Counters are filled only when requested (request |=
 * VRT_STATS_COUNTERS): counting runs the exact-walk instance, ~3x slower than the uncounted
 * frame, so timing alone never asks for it. */
#define VRT_STATS_COUNTERS 1u
typedef struct {
  uint64_t counters[VRT_CNT_COUNT];  /* out (when requested) */
  float kernel_ms;                   /* out */
  uint32_t request;                  /* in: VRT_STATS_* bits */
  float reserved[2];
} vrt_stats;

/* ---- context / device ---------------------------------------------------------------------- */

/* Create a context on the HIP devices of `device_mask` (bit i = device ordinal i):
 * one device renders whole frames; k devices split every whole frame into k block-cyclic bands
 * (ABI v12: device j of the mask renders the 16-row blocks j, j+k, ...; until v11 cyclic rows j,
 * j+k, ...; the volume is replicated on every device: RCCL broadcast from the first device, RCCL
 * communicators over the mask's devices). */
int vrt_create(uint32_t device_mask, vrt_ctx** out);
/* Same over an explicit device list; a device may repeat (rehearses a k-device split on fewer
 * GPUs: the bands and the gather then use device-to-device copies instead of RCCL). */
int vrt_create_devices(const int32_t* devices, int32_t count, vrt_ctx** out);
/* Devices of the context (k), and the ordinal of its i-th device (-1 if out of range). */
int vrt_device_count(const vrt_ctx* ctx);
int vrt_device_ordinal(const vrt_ctx* ctx, int32_t i);
void vrt_destroy(vrt_ctx* ctx);
const char* vrt_last_error(const vrt_ctx* ctx);  /* never NULL; "" when no error */
int vrt_abi_version(void);

/* Copy the volume to device memory (replaces glTexImage3D, main.cpp:315-318): host -> the first
 * device, then a broadcast to the others. The caller keeps ownership of `vol->voxels`. N must be
 * a power of two in [2, 1024]. */
int vrt_upload_volume(vrt_ctx* ctx, const vrt_volume* vol);

/* Same from a DEVICE buffer of N^3 bytes on the context's first GPU (e.g. after an RCCL broadcast
 * of the volume to every GPU of the node by the caller), ordered on `hip_stream`; the context's
 * other devices receive it by broadcast; returns after the copy. */
int vrt_upload_volume_device(vrt_ctx* ctx, const uint8_t* d_voxels, int32_t n, void* hip_stream);

/* Build the _TERRAIN / _GLASS_CUBE / _REFRACTION volume of main.cpp:218-288 directly on the device
 * (bytes identical to vrt_build_scene; only the n*n terrain heightfield is computed on the host)
 * and make it the context's volume, ordered on `hip_stream`; returns after the build. N must be
 * a power of two in [8, 1024]. Replaces the host build + glTexImage3D upload (main.cpp:315-318).
 * Every device of the context builds its own replica (no transfer). */
int vrt_build_scene_device(vrt_ctx* ctx, int32_t scene, int32_t n, uint32_t seed, void* hip_stream);

/* Device pointer of the resident volume (N^3 bytes, canonical layout), e.g. for a broadcast.
 * NULL if none. */
const uint8_t* vrt_volume_device_ptr(const vrt_ctx* ctx);

/* Diagnostic: copy the kernel's device volume to `out` (count >= octants x (N+1)^3, see
 * vrt_volume_octants): per octant o (bit 0: dir.x < 0, bit 1: dir.y < 0, bit 2: dir.z < 0), a padded
 * (N+1)^3 u16 volume = voxel | G << 8 (x fastest; plane N repeats plane 0 with G = 0). Octant
 * layout (N <= 512): G(v) = F(v - s) - 1, F(u) = edge of the largest empty in-volume cube anchored
 * at u extending along s = the octant's step (capped at 64). Single layout (N = 1024): G = the
 * Chebyshev distance to the nearest non-empty voxel or the volume outside, capped at 64.
 * Synchronous. */
int vrt_debug_packed_volume(vrt_ctx* ctx, uint16_t* out, uint64_t count);

/* ABI v5: number of packed volumes of the resident volume (8 octant volumes, or 1 for N = 1024;
 * 0 when none is uploaded). */
int vrt_volume_octants(const vrt_ctx* ctx);

/* ABI v5: skip-distance layout of the NEXT volume upload: 0 = automatic (8 octant volumes for
 * N <= 512, else 1), 1 = one volume with the centred Chebyshev distance (the N = 1024 layout, at
 * any N: tests and A/B timing), 8 = octant volumes where they fit. Images are identical. */
int vrt_set_skip_layout(vrt_ctx* ctx, int32_t octants);

/* ABI v6: certified walks for stats-free colour-only frames (DESIGN.md §6 "Certified walks"): a
 * pixel whose primary outcome and shadow bit provably equal the exact walks' is shaded from a
 * few empty-space jumps; every other pixel (glass hits, near-edge crossings) takes the exact walk,
 * whose shadow rays and air-medium secondary rays are again certified walks when they can be.
 * mode 1 = always, -1 = never (exact walks only), 0 = automatic (default): with the octant layout,
 * certified pixels unless glass makes up more than 1/8 of the resident volume's non-empty voxels
 * (glass pixels pay the certified primary walk before the exact path), certified exact-path rays
 * always. Frames with hit records or counters and textured frames always take the exact walks.
 * Images are identical in every mode. */
int vrt_set_certified(vrt_ctx* ctx, int32_t mode);

/* ABI v6: 1 when the next stats-free colour-only frame tries certified walks for whole pixels,
 * else 0. */
int vrt_certified(const vrt_ctx* ctx);

/* ABI v8 (r02): device timestamps of the async band launches (vrt_render_rows*_async,
 * vrt_render_temporal_rows*_async on the first device): vrt_set_launch_timing(ctx, n) creates
 * timing events for the next n launches (0: off; it synchronises the first device when replacing
 * earlier events), each launch then records its kernel's start and end on the device
 * (hipExtLaunchKernelGGL); vrt_launch_timing waits for the recorded launches, returns the sum of
 * their kernel durations and their count, and frees the events for the next n launches. This is
 * the per-kernel duration a profiler reports, measured in the caller's own timed region. */
int vrt_set_launch_timing(vrt_ctx* ctx, int32_t launches);
int vrt_launch_timing(vrt_ctx* ctx, double* total_ms, uint64_t* launches);

/* ABI v7: heavy-first tile order for stats-free colour-only launches with certified pixels
 * (vrt_certified() == 1) of volumes with glass (DESIGN.md §6 "Tile order"): on = 1 (default),
 * off = 0. ABI v14: 1 is automatic, launches of at least one dispatch round of resident waves
 * (CUs x 4 x 7: 7168 waves, e.g. 1920 x 240 pixels, on MI355X; smaller launches have every tile
 * resident at once, so the order would only cost its bookkeeping), 2 = every launch. Each launch records which of its 16x8 tiles had a pixel on the exact path (glass
 * bounce stacks, near-edge walks; until ABI v8 only bounce stacks); the next launch of the same
 * band (width, rows, row0, row_step) on the same stream dispatches those tiles first, each on the
 * same XCD as before, the last to finish first, so the frame's longest waves start first.
 * Launches on a stream that is being captured into a graph use dispatch order. Every tile is
 * rendered exactly once in any case: images are identical with and without it.
 * ABI v8: the state is a pool allocated by vrt_create (ABI v9: 16 slots of 5 x 65536 words + a
 * header; since v14 5 x 131072 words: launches up to 131072 tiles, i.e. 4096 x 4096 pixels; larger
 * launches use dispatch order), a
 * slot per (band, stream), zeroed on the launch stream when it is (re)assigned. Reassigning the
 * least recently used slot (more than 16 band/stream pairs in use) synchronises the device once
 * (ABI v9: the old stream is never touched; its owner may have destroyed it). */
int vrt_set_tile_order(vrt_ctx* ctx, int32_t on);

/* ABI v9: deferred exact pass for stats-free launches with certified pixels (vrt_certified() == 1):
 * on = 1 (default, automatic) or 2 (always, whatever the band size: tests and A/B timing): the
 * certified pass renders the pixels its certified walks settle and appends the others (glass hits,
 * near-edge walks, textured hits near a texel edge) to a list, in 8 segments by column block of the
 * band (ABI v13; spatially coherent batches); a second kernel on the same stream renders them with
 * the exact path: a wave's own >= 32 pixels as one chunk, the rest 32 to a wave (16 in short bands).
 * It pays when other work overlaps the exact pass and the launch is large: the async band entry
 * points and the device-output frames (frames in flight) use it for bands of at least two rounds of
 * resident waves (CUs x 4 x 7 x 2 waves: 14336, e.g. 1920 x 960 pixels, on MI355X); smaller bands
 * and the synchronous whole-frame calls (vrt_render, vrt_render_frame) keep the in-lane path, except
 * a synchronous colour-only frame (u_Alpha = 1 for vrt_render_frame) of a glass-heavy volume or of
 * >= 8 rounds of resident waves, which is one deferred launch with the exact pass's short-band
 * instance (its in-lane alternative waits on the glass trees, or the long certified pass carries
 * the exact pass's tail; C1 0.330 -> 0.25 ms, C4 0.247 -> 0.21). off =
 * 0: the exact path runs in the pixel's own lane, with the heavy-first tile order
 * (vrt_set_tile_order). Launches over 131072 tiles, and launches on a stream being captured into a
 * graph, use the in-lane path. Images are identical either way. */
int vrt_set_exact_pass(vrt_ctx* ctx, int32_t on);

/* ABI v15: certified bounce trees for stats-free colour-only frames with certified pixels
 * (DESIGN.md §6 "Certified bounce trees"): 1 = automatic (default), 2 = always, 0 = off. A pixel
 * whose primary ray hits glass has its whole bounce tree (voxel.glsl:425-452) walked by certified
 * walks from the certified hits' uncertain origins, the colour folded in the reference's order;
 * any ray whose walk, start or direction could differ from the exact path's sends the pixel to the
 * exact path (deferred or in lane, as above). The certified pass that runs the trees is its own
 * kernel instance (more registers per lane); automatic mode uses it for the volumes whose glass is
 * more than 1/8 of the non-empty voxels, where the automatic certified mode (vrt_set_certified 0)
 * would otherwise render every pixel exactly, so the certified mode is then on for them too; in
 * glass-light volumes the few glass pixels keep the deferred exact path. Images are identical in
 * every mode. */
int vrt_set_cert_trees(vrt_ctx* ctx, int32_t on);

/* Diagnostic: the kernel's RandomizeDirection (voxel.glsl:132-140) for n (dir, pos) float3
 * pairs, out = n float3. Synchronous. */
int vrt_debug_randomize(vrt_ctx* ctx, const float* dir, const float* pos, int32_t n,
                        float randomness, float seed, float* out);

/* Diagnostic: the kernels' fast correctly rounded reciprocal (the hardware reciprocal plus one
 * Newton step) and square root (the hardware square root plus its residual fix) checked against
 * the IEEE division and square root over all 2^32 float bit patterns on the context's first
 * device. out[7]: patterns the kernels take the reciprocal for, mismatches among them (must be 0),
 * mismatches of normal-range patterns with an all-ones significand and of the remaining non-NaN
 * patterns (both take the division), the first mismatching pattern of the first kind (~0 if none),
 * positive patterns the kernels take the square root for, mismatches among them (must be 0).
 * Synchronous. */
int vrt_debug_fast_math(vrt_ctx* ctx, uint64_t* out);

/* Diagnostic (test rehearsal of the multi-GPU path on a one-GPU box): a one-device context takes
 * the k-device path through RCCL with a one-rank communicator (ncclCommInitAll over its device):
 * the volume upload goes through ncclBroadcast (in place) and vrt_render_frame_device through
 * ncclGather of the band into the gather buffer and the strided assembly copy, as with k distinct
 * GPUs. Call once, right after vrt_create with one device; frames are identical either way. */
int vrt_debug_collectives(vrt_ctx* ctx);

/* Synchronous whole-frame render (replaces main.cpp:325-361): writes W*H RGBA floats
 * (alpha = 1, voxel.glsl:451) to the HOST buffer out_rgba. out_hit (W*H records) and stats may
 * be NULL. Hit records or counters run the exact-walk instance; otherwise the fast instance on
 * the context's streams. Each device copies its band straight into the host rows. */
int vrt_render(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* params,
               float* out_rgba, vrt_hit* out_hit, vrt_stats* stats);

/* Asynchronous band render into DEVICE buffers on `hip_stream` (hipStream_t, NULL = default).
 * Renders frame rows row0 + i*row_step for i in [0, rows) at full width; output row i of
 * d_out_rgba / d_out_hit holds frame row row0 + i*row_step. d_out_hit and d_counters
 * (VRT_CNT_COUNT uint64, ACCUMULATED into; the caller zeroes them) may be NULL. Counting uses a
 * per-context replica buffer: at most one counted render per context in flight at a time.
 * No host sync, no allocation: capturable in a hipGraph (the tile order is skipped while the
 * stream is being captured). Runs on the context's first device. */
int vrt_render_rows_async(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* params,
                          int32_t row0, int32_t rows, int32_t row_step,
                          float* d_out_rgba, vrt_hit* d_out_hit, uint64_t* d_counters,
                          void* hip_stream);

/* Pitched form (ABI v4): output row i starts i*pitch pixels after d_out_rgba (pitch >= width),
 * so a band can be written straight into its rows of a whole frame: d_out = frame + row0*width,
 * pitch = row_step*width. vrt_render_rows_async is this with pitch = width. */
int vrt_render_rows_pitched_async(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* params,
                                  int32_t row0, int32_t rows, int32_t row_step, int64_t pitch,
                                  float* d_out_rgba, vrt_hit* d_out_hit, uint64_t* d_counters,
                                  void* hip_stream);

/* ---- textured mode (voxel.glsl without _COLOR_ONLY) --------------------- */
/* With vrt_params.color_only = 0 the kernel shades with the textured material table
 * (voxel.glsl:51-68) and GetColor reads the atlas (:174-182) at GetTextureCoordinate (:167-172)
 * of the hit's face plane, with atlas_size = u_AtlasSize and atlas_texture_size =
 * u_AtlasTextureSize (main.cpp:336-337). Atlas: atlas_size^2 RGBA8 texels, row 0 = bottom (GL
 * t = 0), NEAREST + REPEAT; material slot (texX, texY) covers columns [texX*ts, (texX+1)*ts) and
 * rows [size-(texY+1)*ts, size-texY*ts). atlas_size must be a power of two. The context keeps
 * the atlas: it is uploaded by vrt_upload_atlas, or by any render call whose
 * vrt_params.atlas_rgba is non-NULL and whose bytes (or size) differ from the last upload
 * (compared on the host each call; a synchronous copy when they differ; ABI v8: by content, not
 * by pointer identity). atlas_rgba = NULL renders with the context's atlas: a frame loop uploads
 * once and passes NULL (a non-NULL atlas costs a host compare of its bytes on every call, ~10 us
 * for 256 x 256). Replaces the Atlas texture of main.cpp:187-193. */
int vrt_upload_atlas(vrt_ctx* ctx, const uint8_t* rgba, int32_t atlas_size);

/* ---- temporal filter + RGB8 framebuffer ------------------------------ */
/* The reference stores the ray-traced colour into an RGB8 FBO (FrameBuffer.cpp:8), blends it with
 * the previous filtered frame, color = u_Alpha * new + (1 - u_Alpha) * old (temporal.glsl:18,
 * main.cpp:363-377), into a second RGB8 FBO and swaps the two (main.cpp:391). These entry points
 * run that post-pass fused into the render kernel's epilogue. Pixels are RGBA8 words (R in the
 * low byte, A = 255: the FBOs have no alpha), W x rows, row 0 = bottom. Float -> UNORM8 store:
 * clamp [0,1], x255, round half to even, NaN -> 0 (GL leaves ties/NaN implementation-defined).
 * u_Alpha defaults to 1.0 (res/guis/header.xml:20), which makes the output the quantised frame. */

/* Asynchronous band form on DEVICE buffers, same band/counter/stream rules as
 * vrt_render_rows_async. d_prev_rgba8 holds the band's previous filtered frame and may alias
 * d_cur_rgba8 (each pixel is read before it is written, by the same work-item). d_raw_rgba8
 * (optional) receives the quantised ray-trace frame. */
int vrt_render_temporal_rows_async(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* params,
                                   float alpha, int32_t row0, int32_t rows, int32_t row_step,
                                   const uint32_t* d_prev_rgba8, uint32_t* d_cur_rgba8,
                                   uint32_t* d_raw_rgba8, vrt_hit* d_out_hit, uint64_t* d_counters,
                                   void* hip_stream);

/* Pitched form (ABI v4): row i of d_prev_rgba8, d_cur_rgba8, d_raw_rgba8 and d_out_hit starts
 * i*pitch pixels after the pointer (pitch >= width). With d_prev = d_cur = frame + row0*width and
 * pitch = row_step*width a band filters its rows of one full-frame history in place — the
 * single-GPU frame loop needs no per-band buffers and no assembly copy. */
int vrt_render_temporal_rows_pitched_async(vrt_ctx* ctx, const vrt_camera* cam,
                                           const vrt_params* params, float alpha, int32_t row0,
                                           int32_t rows, int32_t row_step, int64_t pitch,
                                           const uint32_t* d_prev_rgba8, uint32_t* d_cur_rgba8,
                                           uint32_t* d_raw_rgba8, vrt_hit* d_out_hit,
                                           uint64_t* d_counters, void* hip_stream);

/* ABI v11: block-cyclic bands. Band row i is frame row
 *   row0 + (i / row_block) * row_step + i % row_block
 * i.e. blocks of row_block adjacent frame rows, row_step frame rows apart (GPU r of a k-way split
 * with blocks of B rows: row0 = r*B, row_step = k*B, rows = its blocks' rows). row_block is a
 * power of two in [1, 64], and row_step >= row_block unless rows <= row_block; row_block = 1 is the
 * cyclic-row form above. With row_block = 8 an 8x8 pixel wave covers 8 adjacent frame rows, as in
 * a whole frame, instead of 8 rows k apart: the walks of a wave's rays stay coherent (one-GPU
 * rehearsal of GPU 0's band at k = 8: C4 -7 %, C3 -11 % per frame). Everything else
 * (pitch, history, counters, stream, timing) as vrt_render_rows_pitched_async and
 * vrt_render_temporal_rows_pitched_async. */
int vrt_render_blocks_pitched_async(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* params,
                                    int32_t row0, int32_t rows, int32_t row_step, int32_t row_block,
                                    int64_t pitch, float* d_out_rgba, vrt_hit* d_out_hit,
                                    uint64_t* d_counters, void* hip_stream);
int vrt_render_temporal_blocks_pitched_async(vrt_ctx* ctx, const vrt_camera* cam,
                                             const vrt_params* params, float alpha, int32_t row0,
                                             int32_t rows, int32_t row_step, int32_t row_block,
                                             int64_t pitch, const uint32_t* d_prev_rgba8,
                                             uint32_t* d_cur_rgba8, uint32_t* d_raw_rgba8,
                                             vrt_hit* d_out_hit, uint64_t* d_counters,
                                             void* hip_stream);

/* ABI v14: a FRAME BATCH: the same band of `nframes` (1..8) frames in ONE launch, at u_Alpha = 1
 * (each frame's RGB8 store is its output; no history is read), frame f with its own camera
 * cams[f] (same image size) and u_Time params[f].time, written to d_cur_rgba8[f] (and
 * d_raw_rgba8[f] when d_raw_rgba8 is not NULL; pitch
 * pixels per band row in all of them). Band geometry as vrt_render_temporal_blocks_pitched_async;
 * bands of < 8192 rows. A band of a k-way split is 1/k of the frame's waves: below a few dispatch
 * rounds a launch is bound by its longest waves and by the hardware queues that overlap launches,
 * not by the GPU's throughput, and a batch of k frames gives it a whole frame's waves again (the
 * deferred exact pass, the tile order and the grid sizing then see one large launch). Bytes equal
 * nframes single-frame launches' (tests/test_gpu_batch.py). No hit records or counters. A batch
 * of more than 131072 tiles (16x8 pixels) is enqueued as the fewest launches that hold it, of
 * equal frame counts. ABI v15: consecutive frames whose other params fields differ (the day/night
 * cycle moves u_SunDir every frame, main.cpp:346-348) are split into launches of equal fields, in
 * frame order on the stream (before v15: an error). */
int vrt_render_temporal_batch_async(vrt_ctx* ctx, int32_t nframes, const vrt_camera* cams,
                                    const vrt_params* params, int32_t row0, int32_t rows,
                                    int32_t row_step, int32_t row_block, int64_t pitch,
                                    uint32_t* const* d_cur_rgba8, uint32_t* const* d_raw_rgba8,
                                    void* hip_stream);

/* Synchronous frame loop of main.cpp:323-393 with the history and the ray-trace FBO kept in the
 * context: render, filter against the last filtered frame, copy the new filtered frame to the
 * HOST buffer out_rgba8 (W*H*4 bytes). The history starts black and restarts black when the image
 * size changes. stats may be NULL. Each device renders its row band as two interleaved parts on
 * two context-owned streams (one launch's tail overlaps the other's), or as one deferred launch
 * (vrt_set_exact_pass: glass-heavy volumes, large frames); ABI v9: every device's DMA
 * engine writes its band straight into its rows of a pinned staging frame owned by the context
 * (the k copies run in parallel), which is then copied to out_rgba8. */
int vrt_render_frame(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* params, float alpha,
                     uint8_t* out_rgba8, vrt_stats* stats);

/* ABI v8: the same frame for display on the first device, asynchronously. *d_frame receives a
 * device pointer (first GPU) to the new filtered frame, W*H RGBA8 words, row 0 = bottom, owned by
 * the context; hip_stream is made to wait for it, so work the caller enqueues there afterwards
 * (e.g. the texture upload / blit of main.cpp:379-385) sees the frame. The frame stays valid until
 * the fourth later call, which overwrites it only after the work the caller had enqueued on
 * hip_stream before the next call. One device: the frame is rendered straight into that buffer
 * (no copy); several devices: the bands are gathered to the first one over xGMI by ncclGather
 * (rccl.h) and placed into their rows by strided copies. Consecutive frames overlap on the GPU:
 * at u_Alpha = 1 a frame does not read its history and up to four frames are in flight (ABI v9);
 * otherwise part q of a frame waits only for part q of the frame before (its history rows).
 * Returns after the launches; stats may be NULL (then no host sync happens; with stats the call
 * waits for the frame).
 * ABI v9: hip_stream = NULL orders nothing with the caller's streams. The caller then consumes the
 * frame on the stream that produced it (vrt_frame_stream, right after the call): work enqueued
 * there runs after the frame and before the frame that next reuses its buffer (the eighth later
 * call), so no ordering packet crosses streams (with a caller stream, each frame's wait costs
 * ~0.01-0.02 ms of GPU throughput at C3); the host blocks only when it is eight
 * frames ahead of the GPU. */
int vrt_render_frame_device(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* params,
                            float alpha, void* hip_stream, const uint32_t** d_frame,
                            vrt_stats* stats);

/* ABI v9: the HIP stream (hipStream_t) that rendered (or, with several devices, assembled) the last
 * device-output frame of a hip_stream = NULL call, on the first device; NULL before one. */
void* vrt_frame_stream(const vrt_ctx* ctx);

/* "Clear framebuffer" (key F, main.cpp:417-421): the last ray-traced frame becomes the history of
 * the next frame. ABI v9: no buffer changes hands (a device-output frame the caller holds keeps
 * its contents and lifetime). */
int vrt_history_reset(vrt_ctx* ctx);

/* ---- host-side scene harness (mirrors src/main.cpp; no GPU needed) ----------------------- */

enum { VRT_SCENE_TERRAIN = 0, VRT_SCENE_GLASS_CUBE = 1, VRT_SCENE_REFRACTION = 2 };

/* Build-defined seeded heightfield in [0,1) replacing Greet::Noise::GenNoise (main.cpp:185,195);
 * out has n*n floats, index x + z*n. See DESIGN.md "Terrain noise". */
int vrt_terrain_noise(int32_t n, uint32_t seed, float* out);

/* Fill out[n^3] exactly as main.cpp:218-288 does for _TERRAIN / _GLASS_CUBE / _REFRACTION. */
int vrt_build_scene(int32_t scene, int32_t n, uint32_t seed, uint8_t* out);

/* invPV = inverse(P * V) with P = Perspective(aspect, fov_deg, near, far) and
 * V = RotateX(-rot_x) * RotateY(-rot_y) * Translate(-pos)   (main.cpp:67-76, 161). Angles in
 * degrees. Computed in double, rounded to float. */
int vrt_camera_make(const float pos[3], const float rot_deg[3], int32_t width, int32_t height,
                    float fov_deg, float near_plane, float far_plane, vrt_camera* out);

/* u_SunDir from the day/night clock (main.cpp:346-348). */
void vrt_sun_dir(float time_of_day, float day_time, float out[3]);

/* Default params for the bench configs (noise 0, max_ray_length 100, colour-only, time 1). */
void vrt_params_default(vrt_params* out);

/* ABI v8: the row plan of a whole frame of `height` rows over k devices with `parts` interleaved
 * parts each (host arithmetic, no GPU): for band j (device j) and part p, the frame rows
 * row0 + i*row_step (i < rows) that the part renders, written to band-buffer row
 * band_row0 + i*parts. out[(j*parts + p)*4 + 0..3] = {row0, rows, row_step, band_row0}; a band
 * holds ceil((height - j) / k) rows, band row r = frame row j + r*k. Returns the largest band's
 * rows. LEGACY (cyclic rows): since ABI v12 the whole-frame entry points split a frame of
 * k > 1 devices into block-cyclic bands (vrt_block_band_plan) and use this plan only for the
 * interleaved parts of one device's frame (k = 1); kept exported for tests. */
int vrt_band_plan(int32_t height, int32_t k, int32_t parts, int32_t* out);

/* ABI v10: the k strided copies that assemble a frame of `height` rows x `width` pixels of
 * `elem_bytes` each from the k band buffers (band j's rows packed, band row r = frame row j + r*k):
 * the pinned host staging of vrt_render / vrt_render_frame over k devices and the device-frame
 * gather use exactly these. out[j*5 + 0..4] = {destination byte offset, destination pitch, source
 * pitch, row bytes, rows} of one 2-D copy (hipMemcpy2D). Host arithmetic, no GPU; returns k.
 * LEGACY (cyclic rows, as vrt_band_plan): the k > 1 whole-frame paths use vrt_block_copy_plan's
 * copies since ABI v12. Exported for tests (unequal bands when height % k != 0). */
int vrt_band_copy_plan(int32_t width, int32_t height, int32_t k, int32_t elem_bytes, int64_t* out);

/* ABI v12: rows per block of the bands the whole-frame entry points split a frame into over k
 * devices: 1 for k = 1 (the whole frame), 16 for k > 1 (block-cyclic bands). */
int vrt_frame_row_block(int32_t k);

/* ABI v12: the block-cyclic band of every device j < k for blocks of row_block rows (a power of
 * two <= 64): out[j*3 + 0..2] = {row0, rows, row_step}, band row i = frame row
 * row0 + (i / row_block) * row_step + i % row_block (the *_blocks_pitched_async arguments; k = 1:
 * the whole frame). Returns the largest band's rows. Host arithmetic, no GPU. */
int vrt_block_band_plan(int32_t height, int32_t k, int32_t row_block, int32_t* out);

/* ABI v12: the 2-D copies that assemble a frame from k packed block-cyclic band buffers (what
 * vrt_render / vrt_render_frame stage with over k > 1 devices when row_block is
 * vrt_frame_row_block(k)): per band two entries, out[(j*2 + c)*7 + 0..6] = {band j, destination
 * byte offset, destination pitch, source byte offset, source pitch, width bytes, rows} (the band's
 * full blocks, then a short last block; rows = 0 when absent). Returns the number of copies. */
int vrt_block_copy_plan(int32_t width, int32_t height, int32_t k, int32_t row_block, int32_t elem_bytes,
                        int64_t* out);

/* ---- one process per GPU (ABI v12) ------------------------------------------------------------
 * A job of nranks processes, one GPU each (torchrun), each rendering its block-cyclic band of
 * every frame into its own buffers, gathers the bands to rank 0 over RCCL (xGMI) and assembles the
 * frame there — the drop-in's ncclGather path with the ranks in separate processes. */
#define VRT_COMM_ID_BYTES 128
/* A new RCCL unique id (ncclGetUniqueId) into out (>= VRT_COMM_ID_BYTES bytes; rank 0 creates the
 * ids and the job distributes them). Returns VRT_COMM_ID_BYTES. */
int vrt_comm_unique_id(uint8_t* out, int32_t bytes);
/* Join `count` communicators (ids: count x VRT_COMM_ID_BYTES) as `rank` of `nranks` on the
 * context's device (one-device contexts). Blocks until every rank has joined each one, in order.
 * One communicator per lane of frames in flight: a communicator's operations run in issue order,
 * separate ones do not order each other. */
int vrt_comm_join(vrt_ctx* ctx, const uint8_t* ids, int32_t count, int32_t nranks, int32_t rank);
/* ncclGather of `bytes` from d_band on every rank to rank 0's d_gathered (nranks x bytes, rank
 * order; ignored elsewhere) over communicator `comm`, enqueued on hip_stream. */
int vrt_gather_band_async(vrt_ctx* ctx, int32_t comm, const void* d_band, uint64_t bytes, void* d_gathered,
                          void* hip_stream);
/* The frame (height rows of width RGBA8 words, rows frame_pitch words apart) from k gathered
 * block-cyclic bands of row_block rows (band j at d_bands + j * band_rows_cap * width words, band
 * row i = frame row ((i / row_block) * k + j) * row_block + i % row_block): one HIP kernel, one
 * workgroup per frame row, on hip_stream. */
int vrt_assemble_blocks_async(vrt_ctx* ctx, const uint32_t* d_bands, int32_t k, int32_t band_rows_cap,
                              int32_t width, int32_t height, int32_t row_block, uint32_t* d_frame,
                              int64_t frame_pitch, void* hip_stream);
/* RGB8 wire format of a gathered band: the RGBA8 words' A byte is always 255, so a band can cross
 * xGMI as 3 bytes per pixel (25 % fewer bytes into rank 0). vrt_pack_rgb8_async packs `pixels`
 * RGBA8 words (a multiple of 4; 16-byte aligned) into 3-byte pixels (4-byte aligned);
 * vrt_assemble_blocks_rgb8_async is vrt_assemble_blocks_async from such bands (band j at
 * d_bands + j * band_rows_cap * width * 3 bytes; width and frame_pitch multiples of 4), unpacking
 * to RGBA8 words with A = 255. */
int vrt_pack_rgb8_async(vrt_ctx* ctx, const uint32_t* d_rgba8, uint64_t pixels, uint8_t* d_rgb8, void* hip_stream);
int vrt_assemble_blocks_rgb8_async(vrt_ctx* ctx, const uint8_t* d_bands, int32_t k, int32_t band_rows_cap,
                                   int32_t width, int32_t height, int32_t row_block, uint32_t* d_frame,
                                   int64_t frame_pitch, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* VRT_H */
