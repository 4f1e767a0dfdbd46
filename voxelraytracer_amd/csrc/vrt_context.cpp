// vrt_context.cpp — the C-ABI context of include/vrt.h around the kernels of vrt_render.hip.
//
// A context spans the devices of its mask. Every device holds a "shard": a
// replica of the volume in the kernel's packed layout, kLanes lanes of context-owned streams, its
// row band's history / ray-trace / float buffers, counters and the tile-order pool. Whole-frame
// entry points split the frame into cyclic row bands (device j renders rows j, j+k, ...; sky and
// geometry rows balance across devices). Frame f renders on lane f % kLanes: device-output frames
// that do not read their history (u_Alpha = 1) are one launch per band and up to kLanes of them are
// in flight, the next frames' waves filling the slots one frame's longest waves hold; frames that
// run alone or read their history are two interleaved row parts, whose launches overlap each
// other's tails (DESIGN.md §6 "Tail hiding", §8 "Frames in flight"). The reference's single GL
// draw (main.cpp:323-361) becomes k (or 2k) concurrent launches.
// The only exchange is the output: synchronous host outputs are written by each device's DMA
// engine straight into its rows of a pinned staging frame (k links in parallel, no device hop);
// the device-output frame is gathered to the first device with ncclGather over xGMI
// (rccl.h:745). The volume reaches the other devices by ncclBroadcast from the first one.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "vrt.h"
#include "vrt_internal.h"

namespace {

constexpr int kParts = 2;              // interleaved row parts of a frame that runs alone
// Whole frames rotate over kLanes lanes: frame f renders on lane f % kLanes (kParts streams and
// timing events of its own) into history ring slot f % kRing. At u_Alpha = 1 a frame does not read
// its history, so consecutive device-output frames are independent and up to kLanes of them are in
// flight: the light waves of the next frames fill the wave slots one frame's exact-path waves hold
// (C3 0.0618 -> 0.0599 ms per frame on one GPU, C3's band at k = 8 GPUs 0.0416 -> 0.0112 ms;
// profiles/r03_pipe). Such frames are one launch (a second part
// only adds launch overhead once other frames fill the tail); frames that run alone (synchronous
// calls) or read their history (u_Alpha != 1: part q of frame f waits for part q of frame f - 1)
// are kParts interleaved parts, whose launches overlap each other's tails.
constexpr int kLanes = 4;
constexpr int kOrderSlots = 16;        // tile-order buffers per device (band geometry x stream)
constexpr uint32_t kOrderMaxTiles = 1u << 17;  // launches up to 131072 16x8 tiles (e.g. 7 frames of a 7-way 4K band)
constexpr size_t kOrderSlotWords = vrt::kOrdHdr + 5u * size_t(kOrderMaxTiles) + 2u * vrt::kOrdClasses;  // KArgs::order
// KArgs::defer: two sets of segment counters, then the list: a pixel per word, 8 segments of
// ceil(tiles / 8) tiles' pixels each. Allocated per tile-order slot at its first deferred launch,
// sized for that band (a 1080p band: 8.3 MB; until r03 every slot was sized for 65 536 tiles up
// front, 537 MB per device).
// tiles of the largest segment: a column block of the band (tile columns tx * 8 / tiles_x)
uint32_t defer_seg_tiles(uint32_t tiles, uint32_t tiles_x) {
  return (tiles_x + vrt::kOrdClasses - 1u) / vrt::kOrdClasses * (tiles / tiles_x);
}
size_t defer_words(uint32_t tiles, uint32_t tiles_x) {
  return vrt::kDeferHdr + size_t(vrt::kOrdClasses) * defer_seg_tiles(tiles, tiles_x) * vrt::kWgThreads;
}
#if (defined(VRT_DEV_NOQUERY) || defined(VRT_DEV_NOCONSUME) || defined(VRT_DEV_NOCSWAIT)) && \
    !defined(VRT_DIAGNOSTIC_BUILD)
#error "VRT_DEV_* are diagnostic knobs of make variant builds"
#endif
// Filtered frames rotate through kRing buffers: frame f reads ring[(f-1) % kRing] (the temporal
// history) and writes ring[f % kRing]. A device-output frame (vrt_render_frame_device) is handed
// to the caller as its ring buffer and stays valid until the fourth later call, with no copy. Eight
// slots for four lanes: frame f overwrites the slot of frame f - 8, whose consumption the caller
// had enqueued well before frame f - 4 (frame f's predecessor on its lane) ends, so the wait for
// it costs nothing in the steady state (with four slots every frame waited for its lane
// predecessor's consumption through two command-processor hops: C3 0.0719 vs 0.0596 ms per frame).
constexpr int kRing = 8;
static_assert(kRing % kLanes == 0, "a ring slot is always written from the same lane");

struct OrderSlot {
  int32_t width = 0, rows = 0, row0 = 0, row_step = 0, row_blk_sh = 0;
  int32_t nframes = 1;         // frames per launch (frame batches)
  hipStream_t stream = nullptr;
  uint32_t* d = nullptr;       // kOrderSlotWords words inside the shard's pool
  bool used = false;
  uint64_t epoch = 0, tick = 0;
  uint64_t defer_epoch = 0;    // deferred-pass launches since the slot's counters were zeroed
  bool last_defer = false;     // the slot's last launch was a deferred-pass launch
  uint32_t* defer = nullptr;   // the deferred pass's counters + list (lazily allocated)
  size_t defer_cap = 0;        // its words
  uint32_t* h_batches = nullptr;  // host-mapped: an earlier exact pass's batch count (~0u: none)
  uint32_t* d_batches = nullptr;  // its device address
  // end of the slot's last launch (recorded once the pool is under pressure, see acquire_slot):
  // evicting the slot waits for it instead of the whole device
  hipEvent_t ev_last = nullptr;
  bool ev_last_valid = false;
};

struct Shard {
  int device = 0;
  uint32_t wave_slots = 7168;  // resident waves of the certified pass: CUs x 4 SIMDs x 7
  // volume: canonical N^3, distance scratch, the kernel's packed octant volumes
  uint8_t* d_vox = nullptr;
  uint8_t* d_tmp = nullptr;
  uint16_t* d_vox_pad = nullptr;
  int32_t n = 0, octants = 0;
  bool cert_auto = true;   // automatic certified-pixel choice for the resident volume
  bool has_glass = true;   // the resident volume has glass (bounce stacks; tile order)
  unsigned long long* d_vstats = nullptr;  // glass and non-empty voxel counts
  // counters
  unsigned long long* d_cnt = nullptr;      // VRT_CNT_COUNT totals of a synchronous render
  unsigned long long* d_cnt_rep = nullptr;  // kCntReplicas x VRT_CNT_COUNT, kept zeroed
  // whole-frame lanes: streams, and per lane the events of its last frame's launches
  hipStream_t ls[kLanes][kParts] = {};
  hipEvent_t ev_done[kLanes][kParts] = {};
  int lane_parts[kLanes] = {};       // launches of the lane's last frame (0: none)
  int slot_reader[kRing] = {};       // lane + 1 of the frame that read slot s as its history (0: none)
  hipStream_t gs = nullptr;          // gather / assembly / host-copy stream
  hipEvent_t ev_gs = nullptr;        // marker on gs (volume upload ordering, gather done)
  hipEvent_t ev_band_read[kRing] = {};  // gs has read ring slot s (device-output gather)
  bool band_read_valid[kRing] = {};
  // GPU time of each launch of the last synchronous frame: recorded when the kernel starts /
  // ends on the device
  hipEvent_t ev_kbeg[kParts] = {}, ev_kend[kParts] = {};
  bool timed[kParts] = {};
  // this device's row band of the whole-frame buffers (band_cap rows x width)
  uint32_t* d_ring[kRing] = {};      // filtered bands (history ring)
  uint32_t* d_rawbuf[kRing] = {};    // quantised ray-trace band of frame f (rayTrace FBO; key F)
  size_t hist_pixels = 0;
  float4* d_out = nullptr;     // vrt_render's float band
  vrt_hit* d_hit = nullptr;
  size_t out_pixels = 0;
  // textured mode's atlas (RGBA8 words)
  uint32_t* d_atlas = nullptr;
  int32_t atlas_size = 0;
  // heavy-first tile order, and the deferred exact pass's lists (same slots)
  uint32_t* d_order_pool = nullptr;
  OrderSlot order[kOrderSlots];
  uint64_t order_tick = 0;
  uint32_t order_assigned = 0;  // (band, stream) pairs assigned to slots so far
};

}  // namespace

struct vrt_ctx {
  std::vector<Shard> sh;
  bool distinct = true;                 // devices pairwise distinct: RCCL communicators exist
  bool coll1 = false;                   // one device through the RCCL path (vrt_debug_collectives)
  std::vector<ncclComm_t> comms;
  int32_t layout_req = 0;               // vrt_set_skip_layout
  int32_t cert_req = 0;                 // vrt_set_certified
  int32_t tree_req = 1;                 // vrt_set_cert_trees
  int tile_order = 1;                   // vrt_set_tile_order: 0 off, 1 automatic, 2 always
  int32_t exact_pass = 1;               // vrt_set_exact_pass: 0 off, 1 automatic, 2 always
  // vrt_set_launch_timing: timing events for the async band launches' device start / end
  // timestamps (2 per launch, created up front), and how many are in use since the last read
  std::vector<hipEvent_t> lt_ev;
  size_t lt_used = 0;
  std::vector<uint8_t> atlas_host;      // bytes of the last atlas upload (a params pointer is
                                        // re-uploaded when its bytes differ, not by identity)
  int32_t hist_w = 0, hist_h = 0;       // image size of the resident whole-frame history
  uint64_t fk = 0;                      // frames rendered into the resident history
  bool raw_is_cur[kRing] = {};          // frame in slot s had u_Alpha = 1: its raw frame = ring[s]
  bool reset_pending = false;           // vrt_history_reset: the next frame's history is the raw frame
  uint32_t* d_gather = nullptr;         // first device: k x band_cap x width words (ncclGather)
  size_t hist_pixels_gather = 0;
  uint32_t* d_frames[kRing] = {};       // first device, k > 1: assembled frames
  // caller stream, device-output frames: E_f = ev_consumed[f % kRing], recorded at call f, marks
  // the caller's work enqueued before call f (its consumption of frames <= f - 1)
  hipEvent_t ev_consumed[kRing] = {};
  bool consumed_valid[kRing] = {};
  hipEvent_t ev_gathered = nullptr;     // first device: the last device-output frame is assembled
  // device-output frames with no caller stream (vrt_frame_stream): the stream that rendered (or
  // assembled) the last frame, and per ring slot the end of the frame rendered into it (host
  // back-pressure: at most kRing frames ahead)
  hipStream_t frame_stream = nullptr;
  hipEvent_t ev_slot[kRing] = {};
  bool slot_valid[kRing] = {};
  void* h_stage = nullptr;              // pinned host staging of synchronous frames (k bands in)
  size_t h_stage_bytes = 0;
  // ABI v12: this process's rank of a one-process-per-GPU job (vrt_comm_join): one RCCL
  // communicator per lane, so that frames in flight on different lane streams gather without
  // ordering each other (a communicator's operations run in issue order)
  std::vector<ncclComm_t> rank_comms;
  int32_t rank_nranks = 0, rank_id = -1;
  std::string err;
};

namespace {

int fail(vrt_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int hip_fail(vrt_ctx* c, hipError_t e, const char* what) {
  return fail(c, VRT_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

int nccl_fail(vrt_ctx* c, ncclResult_t r, const char* what) {
  return fail(c, VRT_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}

#define VRT_HIP(ctx, call)                                   \
  do {                                                       \
    hipError_t e_ = (call);                                  \
    if (e_ != hipSuccess) return hip_fail((ctx), e_, #call); \
  } while (0)

#define VRT_NCCL(ctx, call)                                    \
  do {                                                         \
    ncclResult_t r_ = (call);                                  \
    if (r_ != ncclSuccess) return nccl_fail((ctx), r_, #call); \
  } while (0)

// The caller's current device is restored when an entry point returns (entry points switch
// between the context's devices).
struct DeviceGuard {
  int dev = -1;
  DeviceGuard() { (void)hipGetDevice(&dev); }
  ~DeviceGuard() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
};

// Cyclic-row bands (ABI v8/v10 plans): band j holds frame rows j, j + k, ...
int32_t cyc_band_rows(int32_t height, int32_t k, int32_t j) { return j < height ? (height - j + k - 1) / k : 0; }

// Whole frames over k > 1 devices (ABI v12): block-cyclic bands of kFrameRowBlock adjacent rows,
// band j = blocks j, j + k, ... (band row i = frame row ((i / B) k + j) B + i % B), one launch per
// band and frame, as bench.py's one-process-per-GPU split (tiles.block_band_spec): an 8x8 wave of
// a band covers 8 adjacent frame rows as in the whole frame, so its walks stay coherent (slowest
// of 8 bands: C3 0.0150 -> 0.0139, C4 0.0274 -> 0.0229 ms per frame against cyclic rows,
// profiles/r03_s45, r03_s54). One device renders the whole frame (B = 1, kParts parts).
constexpr int32_t kFrameRowBlock = 16;
constexpr int32_t kFrameRowBlockSh = 4;
static_assert((1 << kFrameRowBlockSh) == kFrameRowBlock, "row block is 2^sh");
struct BandGeom {
  int32_t row0, rows, row_step, sh;
};
BandGeom block_band(int32_t height, int32_t k, int32_t block, int32_t j) {
  if (k == 1) return BandGeom{0, height, 1, 0};
  int32_t sh = 0;
  while ((1 << sh) < block) ++sh;
  const int32_t nb = (height + block - 1) / block;
  const int32_t own = j < nb ? (nb - j + k - 1) / k : 0;
  int32_t rows = own * block;
  if (own > 0 && (nb - 1) % k == j) rows -= nb * block - height;
  return BandGeom{j * block, rows, k * block, sh};
}
// rows of the largest of the k bands (band 0 unless it also owns the short last block)
int32_t largest_band(int32_t height, int32_t k, int32_t block) {
  int32_t m = 0;
  for (int32_t j = 0; j < k; ++j) m = std::max(m, block_band(height, k, block, j).rows);
  return m;
}
int32_t frame_block(int32_t k) { return k > 1 ? kFrameRowBlock : 1; }
int32_t band_rows(int32_t height, int32_t k, int32_t j) { return block_band(height, k, frame_block(k), j).rows; }
// rows of the largest band (band 0's): every band buffer and the gather's per-device slice
int32_t band_cap(int32_t height, int32_t k) {
  if (k == 1) return height;
  const int32_t nb = (height + kFrameRowBlock - 1) / kFrameRowBlock;
  return (nb + k - 1) / k * kFrameRowBlock;
}

// The 2-D copies that place band j (its rows packed at `row` bytes each) into its frame rows:
// cyclic rows (block 1) are one copy of `rows` rows k rows apart; block-cyclic bands one copy of
// the band's full blocks (block x row bytes each, k blocks apart) and one of a short last block.
// Staging to the host and the device-to-device assembly use exactly these (vrt_block_copy_plan).
struct BandCopy {
  size_t dst_off, dst_pitch, src_off, src_pitch, width, rows;
};
int band_copies(int32_t w, int32_t h, int32_t k, int32_t block, int32_t j, size_t elem, BandCopy out[2]) {
  const size_t row = size_t(w) * elem;
  if (block == 1) {
    out[0] = BandCopy{size_t(j) * row, size_t(k) * row, 0, row, row, size_t(cyc_band_rows(h, k, j))};
    return out[0].rows ? 1 : 0;
  }
  const BandGeom g = block_band(h, k, block, j);
  const size_t full = size_t(g.rows) / size_t(block), rest = size_t(g.rows) % size_t(block);
  int n = 0;
  if (full) out[n++] = BandCopy{size_t(j) * block * row, size_t(k) * block * row, 0, size_t(block) * row,
                                size_t(block) * row, full};
  if (rest) out[n++] = BandCopy{(full * size_t(k) + size_t(j)) * size_t(block) * row, rest * row,
                                full * size_t(block) * row, rest * row, rest * row, 1};
  return n;
}

// Part p of band j: frame rows (j + p k) + i (k P), band rows p + i P.
struct PartRows {
  int32_t row0, rows, row_step, band_row0;
};
PartRows part_rows(int32_t height, int32_t k, int32_t parts, int32_t j, int32_t p) {
  const int32_t hb = cyc_band_rows(height, k, j);
  return PartRows{j + p * k, hb > p ? (hb - p + parts - 1) / parts : 0, k * parts, p};
}

void shard_free(Shard& s) {
  (void)hipSetDevice(s.device);
  std::vector<void*> bufs = {(void*)s.d_vox, (void*)s.d_tmp, (void*)s.d_vox_pad, (void*)s.d_vstats,
                             (void*)s.d_cnt, (void*)s.d_cnt_rep, (void*)s.d_out, (void*)s.d_hit,
                             (void*)s.d_atlas, (void*)s.d_order_pool};
  for (OrderSlot& o : s.order) {
    bufs.push_back(o.defer);
    if (o.h_batches) (void)hipHostFree(o.h_batches);
    if (o.ev_last) (void)hipEventDestroy(o.ev_last);
  }
  for (int r = 0; r < kRing; ++r) {
    bufs.push_back(s.d_ring[r]);
    bufs.push_back(s.d_rawbuf[r]);
  }
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  std::vector<hipEvent_t> evs = {s.ev_gs};
  for (int q = 0; q < kParts; ++q) {
    evs.push_back(s.ev_kbeg[q]);
    evs.push_back(s.ev_kend[q]);
  }
  for (int l = 0; l < kLanes; ++l)
    for (int q = 0; q < kParts; ++q) evs.push_back(s.ev_done[l][q]);
  for (int r = 0; r < kRing; ++r) evs.push_back(s.ev_band_read[r]);
  for (hipEvent_t e : evs)
    if (e) (void)hipEventDestroy(e);
  for (int l = 0; l < kLanes; ++l)
    for (int q = 0; q < kParts; ++q)
      if (s.ls[l][q]) (void)hipStreamDestroy(s.ls[l][q]);
  if (s.gs) (void)hipStreamDestroy(s.gs);
  s = Shard();
}

hipError_t shard_init(Shard& s, int device) {
  s.device = device;
  hipError_t e = hipSetDevice(device);
  int cus = 0;
  if (e == hipSuccess && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
      cus > 0)
    s.wave_slots = uint32_t(cus) * 4u * 7u;
  const size_t rep_bytes = sizeof(unsigned long long) * vrt::kCntReplicas * VRT_CNT_COUNT;
  const size_t pool_words = size_t(kOrderSlots) * kOrderSlotWords;
  // ordering markers without timestamps (timing events make the command processor stamp and
  // flush around them: ~20 us gaps between the launches of a stream, measured)
  // HIP deals streams to its hardware queues (GPU_MAX_HW_QUEUES, 4 by default) in creation order:
  // the lanes' first streams first, so that frames in flight land on distinct queues
  for (int q = 0; q < kParts; ++q)
    for (int l = 0; l < kLanes && e == hipSuccess; ++l) {
      e = hipStreamCreateWithFlags(&s.ls[l][q], hipStreamNonBlocking);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&s.ev_done[l][q], hipEventDisableTiming);
    }
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s.gs, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&s.ev_gs, hipEventDisableTiming);
  for (int r = 0; r < kRing && e == hipSuccess; ++r)
    e = hipEventCreateWithFlags(&s.ev_band_read[r], hipEventDisableTiming);
  for (int q = 0; q < kParts && e == hipSuccess; ++q) {
    e = hipEventCreate(&s.ev_kbeg[q]);
    if (e == hipSuccess) e = hipEventCreate(&s.ev_kend[q]);
  }
  if (e == hipSuccess) e = hipMalloc(&s.d_cnt, sizeof(unsigned long long) * VRT_CNT_COUNT);
  if (e == hipSuccess) e = hipMalloc(&s.d_cnt_rep, rep_bytes);
  if (e == hipSuccess) e = hipMemset(s.d_cnt_rep, 0, rep_bytes);
  if (e == hipSuccess) e = hipMalloc(&s.d_order_pool, pool_words * sizeof(uint32_t));
  for (int i = 0; i < kOrderSlots && e == hipSuccess; ++i) s.order[i].d = s.d_order_pool + size_t(i) * kOrderSlotWords;
  return e;
}

// The stream of the shard's one-at-a-time work (volume upload, passes, broadcast): lane 0's first
hipStream_t main_stream(const Shard& s) { return s.ls[0][0]; }

int upload_atlas(vrt_ctx* ctx, const uint8_t* rgba, int32_t size) {
  if (!rgba || size < 1 || size > 8192 || (size & (size - 1)) != 0)
    return fail(ctx, VRT_ERR_INVALID, "atlas edge must be a power of two in [1, 8192]");
  const size_t bytes = size_t(size) * size * 4;
  for (Shard& s : ctx->sh) {
    VRT_HIP(ctx, hipSetDevice(s.device));
    if (s.atlas_size != size) {
      if (s.d_atlas) (void)hipFree(s.d_atlas);
      s.d_atlas = nullptr;
      s.atlas_size = 0;
      if (hipMalloc(&s.d_atlas, bytes) != hipSuccess) return fail(ctx, VRT_ERR_OOM, "hipMalloc atlas");
    }
    VRT_HIP(ctx, hipMemcpy(s.d_atlas, rgba, bytes, hipMemcpyHostToDevice));
    s.atlas_size = size;
  }
  ctx->atlas_host.assign(rgba, rgba + bytes);
  return VRT_OK;
}

int check_render_args(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* p) {
  if (!cam || !p) return fail(ctx, VRT_ERR_INVALID, "null camera or params");
  if (!ctx->sh[0].d_vox_pad) return fail(ctx, VRT_ERR_NO_VOLUME, "no volume uploaded");
  if (cam->width <= 0 || cam->height <= 0 || cam->width > 32768 || cam->height > 32768)
    return fail(ctx, VRT_ERR_INVALID, "bad image size");
  if (!p->color_only) {  // textured mode: the context's atlas (uploaded here when it changes)
    const size_t abytes = p->atlas_size > 0 ? size_t(p->atlas_size) * size_t(p->atlas_size) * 4 : 0;
    if (p->atlas_rgba && (p->atlas_size != ctx->sh[0].atlas_size || abytes != ctx->atlas_host.size() ||
                          std::memcmp(p->atlas_rgba, ctx->atlas_host.data(), abytes) != 0)) {
      const int st = upload_atlas(ctx, p->atlas_rgba, p->atlas_size);
      if (st != VRT_OK) return st;
    }
    if (!ctx->sh[0].d_atlas || p->atlas_size != ctx->sh[0].atlas_size)
      return fail(ctx, VRT_ERR_INVALID, "textured mode needs an atlas of atlas_size (vrt_upload_atlas)");
    if (p->atlas_texture_size <= 0) return fail(ctx, VRT_ERR_INVALID, "atlas_texture_size must be > 0");
  }
  if (p->max_reflections < 0 || p->max_transparencies < 0 ||
      p->max_reflections + p->max_transparencies + 1 > vrt::kMaxStack)
    return fail(ctx, VRT_ERR_UNSUPPORTED, "max_reflections + max_transparencies must be <= 16");
  return VRT_OK;
}

vrt::KArgs make_args(const vrt_ctx* ctx, const Shard& s, const vrt_camera* cam, const vrt_params* p,
                     int32_t row0, int32_t rows, int32_t row_step) {
  vrt::KArgs a;
  std::memcpy(a.inv_pv, cam->inv_pv, sizeof(a.inv_pv));
  std::memcpy(a.sun, p->sun_dir, sizeof(a.sun));
  a.sky_sy = std::fmax(p->sun_dir[1], 0.0f);  // GLSL max(x, 0) with fmaxf's NaN rule, as gmax
  // normalize(u_SunDir) exactly as the kernel's normalize3 (IEEE single ops, no contraction)
  const float sx = p->sun_dir[0], sy = p->sun_dir[1], sz = p->sun_dir[2];
  const float inv = 1.0f / std::sqrt(sx * sx + sy * sy + sz * sz);
  a.sun_n[0] = sx * inv;
  a.sun_n[1] = sy * inv;
  a.sun_n[2] = sz * inv;
  for (int i = 0; i < 3; ++i) a.sun_rcp[i] = 1.0f / a.sun_n[i];
  a.time = p->time;
  a.ray_noise = p->ray_noise;
  a.refl_noise = p->reflection_noise;
  a.refr_noise = p->refraction_noise;
  a.max_len = p->max_ray_length;
  a.n = s.n;
  a.fn = float(s.n);
  a.width = cam->width;
  a.height = cam->height;
  a.rcp_w = 1.0f / float(cam->width);
  a.rcp_h = 1.0f / float(cam->height);
  a.row0 = row0;
  a.rows = rows;
  a.row_step = row_step;
  a.row_blk_sh = 0;
  a.pitch = cam->width;
  a.ostride = s.octants == 8 ? uint32_t(uint64_t(s.n + 1) * (s.n + 1) * (s.n + 1) * sizeof(uint16_t)) : 0u;
  a.max_refl = p->max_reflections;
  a.max_transp = p->max_transparencies;
  a.textured = p->color_only ? 0 : 1;
  a.atlas_size = p->color_only ? 1 : p->atlas_size;
  a.atlas_tex_size = p->atlas_texture_size;
  a.atlas = s.d_atlas;
  a.alpha = 1.0f;
  a.prev = nullptr;
  a.cur = nullptr;
  a.raw = nullptr;
  // automatic mode: certified pixels unless glass dominates the volume, where certified bounce
  // trees (automatic: exactly those volumes) settle the glass pixels instead
  const bool trees = ctx->tree_req == 2 || (ctx->tree_req == 1 && !s.cert_auto);
  a.cert = s.octants != 8 || ctx->cert_req < 0 ? 0 : (ctx->cert_req > 0 || s.cert_auto || trees ? 2 : 1);
  a.tree = a.cert == 2 && p->color_only && trees ? 1 : 0;
  a.tiles_x = uint32_t((a.width + vrt::kTileW - 1) / vrt::kTileW);
  a.tiles = a.tiles_x * uint32_t((a.rows + vrt::kTileH - 1) / vrt::kTileH);
  a.order = nullptr;
  a.ord_r = a.ord_w = a.ctr_r = a.ctr_w = a.ctr_z = a.ord_q = 0;
  a.defer = nullptr;
  a.defer_e = a.defer_seg = 0;
  a.exact_fat = 0;
  a.exact_grid = 0;
  a.batches_out = nullptr;
  a.nframes = 1;
  a.frame_tiles = a.tiles;
  std::memset(a.fb, 0, sizeof(a.fb));
  return a;
}

// The tile-order slot of this launch's band and stream, from the shard's pool (no allocation, no
// host sync in the steady state). A slot stays with its (band, stream): launches on one stream are
// ordered, so no marker is needed per launch while the pool has room (a frame loop uses one slot per
// lane). Reassigning the least recently used slot to another band or stream (more pairs than
// kOrderSlots) must first wait for the old stream's last launch with the slot, and that stream may
// already have been destroyed by its owner, so nothing can be recorded on it then: once half the
// pool has been assigned, every launch with a slot records the slot's ev_last after it
// (slot_launched), and eviction waits for that event; a slot evicted before any such record (the
// pool filled in one burst) falls back to a device synchronisation. Then the slot is zeroed on this
// stream (no heavy tiles yet). Not while the stream is being captured into a graph (a replayed node
// would reuse one list / counter set): dispatch order then.
OrderSlot* acquire_slot(Shard& s, const vrt::KArgs& a, hipStream_t st) {
  if (a.tiles == 0 || a.tiles > kOrderMaxTiles) return nullptr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return nullptr;
  OrderSlot* slot = nullptr;
  for (auto& o : s.order)
    if (o.used && o.width == a.width && o.rows == a.rows && o.row0 == a.row0 && o.row_step == a.row_step &&
        o.row_blk_sh == a.row_blk_sh && o.nframes == a.nframes && o.stream == st)
      slot = &o;
  if (!slot) {
    slot = &s.order[0];
    for (auto& o : s.order)
      if (!o.used || (slot->used && o.tick < slot->tick)) slot = &o;
    if (slot->used && slot->stream != st) {
      const hipError_t e = slot->ev_last_valid ? hipEventSynchronize(slot->ev_last) : hipDeviceSynchronize();
      if (e != hipSuccess) return nullptr;
    }
    slot->ev_last_valid = false;
    ++s.order_assigned;
    // zero the list counters, the wave counters and both rank sets (no heavy tiles yet)
    if (hipMemsetAsync(slot->d, 0, (vrt::kOrdHdr + size_t(3) * a.tiles) * sizeof(uint32_t), st) != hipSuccess)
      return nullptr;
    slot->width = a.width;
    slot->rows = a.rows;
    slot->row0 = a.row0;
    slot->row_step = a.row_step;
    slot->row_blk_sh = a.row_blk_sh;
    slot->nframes = a.nframes;
    slot->stream = st;
    slot->epoch = 0;
    slot->last_defer = false;
    slot->used = true;
  }
  slot->tick = ++s.order_tick;
  return slot;
}

// Per-launch state of a stats-free launch from its slot: the deferred exact pass's mask buffer
// (certified colour-only launches, vrt_set_exact_pass), else the heavy-first tile order.
// allow_defer: false for frames that run alone (synchronous calls): there the exact pass's
// latency after the certified pass is the frame's (C3 0.198 vs 0.076 ms per synchronous frame),
// while frames in flight hide it. The deferral also needs a launch of at least two rounds of the
// certified pass's resident waves: on smaller bands the exact pass's latency (its longest waves
// are the glass pixels' bounce stacks) follows a short certified pass on the same stream and
// bounds the band's frame rate (C3's band at k = 4 / 8 GPUs: 0.025 / 0.0235 ms per frame deferred,
// 0.0155 / 0.0114 in-lane; the whole frame: 0.0445 deferred, 0.060 in-lane; C4's band at k = 8,
// 16 200 waves: 0.0281 deferred, 0.0297 in-lane; profiles/r03_s18, r03_s19).
// After a launch with slot `o` on st: under pool pressure, mark its end for a later eviction.
void slot_launched(Shard& s, OrderSlot* o, hipStream_t st) {
  if (!o || s.order_assigned * 2u < uint32_t(kOrderSlots)) return;
  if (!o->ev_last && hipEventCreateWithFlags(&o->ev_last, hipEventDisableTiming) != hipSuccess) {
    o->ev_last = nullptr;
    return;
  }
  o->ev_last_valid = hipEventRecord(o->ev_last, st) == hipSuccess;
}

// A frame that runs alone (synchronous calls) with the deferred exact pass, as one launch with the
// exact pass's short-band instance: where the in-lane alternative's long waves are the frame
// (glass-heavy volumes: every lane holds its bounce tree) or the certified pass is long enough to
// carry the exact pass's ~50 us tail (>= 8 rounds of resident waves); frames of at least two rounds
// (the deferral's own bound, launch_state_begin) within one list slot. Synchronous frames, device
// timestamps: C1 0.330 -> 0.252 ms, C4 0.247 -> 0.212; C3 0.101 -> 0.103 and C2 0.129 -> 0.146
// stay in lane, as two interleaved parts (profiles/r06_s12).
bool lone_defers(const vrt_ctx* ctx, const Shard& s, const vrt::KArgs& a) {
  const uint32_t waves = a.tiles * uint32_t(vrt::kWgWaves);
  return ctx->exact_pass > 0 && a.cert == 2 && !a.textured && a.rows < 8192 && a.tiles <= kOrderMaxTiles &&
         waves >= 2u * s.wave_slots && (!s.cert_auto || waves >= 8u * s.wave_slots);
}

OrderSlot* launch_state_begin(const vrt_ctx* ctx, Shard& s, vrt::KArgs& a, hipStream_t st, bool allow_defer,
                              bool lone = false) {
  // (the deferred list packs a pixel as frame | band row | column in 3 | 13 | 16 bits)
  const bool defer = allow_defer && ctx->exact_pass > 0 && a.cert == 2 && a.rows < 8192 &&
                     (ctx->exact_pass == 2 || a.tiles * uint32_t(vrt::kWgWaves) >= 2u * s.wave_slots);
  // the tile order only where it pays: glass in the volume (without it the order gains nothing:
  // C2 ±0, C4 +5 %, profiles/r02_s14_tileorder) and certified pixels (glass-heavy volumes, where
  // every tile is heavy, keep dispatch order: C1 +3.4 %)
  // Nor for launches below one dispatch round of waves (VRT_ORD_MIN_ROUNDS): all of their tiles are
  // resident at once, so an order only costs its list reads and bookkeeping (C3's 8-way bands
  // in flight: rank 7 0.0078 -> 0.0072, rank 6 0.0127 -> 0.0105 ms per frame, profiles/r05_s14)
  const bool order = !defer && ctx->tile_order != 0 && !a.textured && a.cert == 2 && s.has_glass &&
                     (ctx->tile_order == 2 ||
                      a.tiles * uint32_t(vrt::kWgWaves) >= uint32_t(VRT_ORD_MIN_ROUNDS) * s.wave_slots);
  if (!defer && !order) return nullptr;
  OrderSlot* slot = acquire_slot(s, a, st);
  if (!slot) return nullptr;
  if (defer) {  // both counter sets zeroed whenever the slot's previous launch was not one
    const size_t need = defer_words(a.tiles, a.tiles_x);
    if (slot->defer_cap < need) {  // first deferred launch of this band on the slot (or a larger band)
      // earlier launches with the slot run on st (its stream) and may still read the old list
      if (slot->defer && (hipStreamSynchronize(st) != hipSuccess || hipFree(slot->defer) != hipSuccess)) return slot;
      slot->defer = nullptr;
      slot->defer_cap = 0;
      if (hipMalloc(&slot->defer, need * sizeof(uint32_t)) != hipSuccess) {
        slot->defer = nullptr;
        return slot;  // no list: the launch keeps the exact path in lane
      }
      slot->defer_cap = need;
      slot->last_defer = false;
    }
    uint32_t* d = slot->defer;
    if (!slot->last_defer) {
      if (hipMemsetAsync(d, 0, vrt::kDeferHdr * sizeof(uint32_t), st) != hipSuccess) return slot;
      slot->defer_epoch = 0;
    }
    a.defer = d;
    a.defer_e = uint32_t(slot->defer_epoch & 1u);
    a.defer_seg = defer_seg_tiles(a.tiles, a.tiles_x) * uint32_t(vrt::kWgThreads);
    // bands of under 4 rounds: the exact pass's latency follows a short certified pass
    a.exact_fat = !a.textured && (lone || a.tiles * uint32_t(vrt::kWgWaves) < 4u * s.wave_slots) ? 1 : 0;
    if (VRT_EXACT_GRID_ADAPT && !a.exact_fat) {
      const uint32_t div = a.textured ? vrt::kDeferGridDiv : vrt::kDeferGridDivColor;  // launch_render's
      // the grid from an earlier frame's batch count on this slot (frames in flight: a few frames
      // old) plus a margin; a larger frame loops its workgroups over the rest. Idle workgroups
      // are not free: each waits for a register and LDS slot among the next frames' waves. Not for
      // short bands, whose frame time is this pass's span (C4 8-way band 0.0196 -> 0.0200 ms with
      // it, profiles/r04_s26)
      if (!slot->h_batches) {
        void* h = nullptr;
        if (hipHostMalloc(&h, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
          slot->h_batches = static_cast<uint32_t*>(h);
          *slot->h_batches = ~0u;
          void* d = nullptr;
          if (hipHostGetDevicePointer(&d, h, 0) == hipSuccess) slot->d_batches = static_cast<uint32_t*>(d);
        }
      }
      if (slot->d_batches) {
        const uint32_t full = std::max(64u, a.tiles * uint32_t(vrt::kWgWaves) / div);
        const uint32_t prev = *static_cast<volatile uint32_t*>(slot->h_batches);
        a.batches_out = slot->d_batches;
        if (prev != ~0u) a.exact_grid = std::min(full, std::max(64u, prev + prev / 4u + 64u));
      }
    }
    slot->defer_epoch++;
    slot->last_defer = true;
    return slot;
  }
  slot->last_defer = false;
  a.order = slot->d;
  a.ord_r = uint32_t(slot->epoch & 1u);
  a.ord_w = a.ord_r ^ 1u;
  a.ctr_r = uint32_t(slot->epoch % 3u);
  a.ctr_w = (a.ctr_r + 1u) % 3u;
  a.ctr_z = (a.ctr_r + 2u) % 3u;
  a.ord_q = vrt::ord_q_for(a.tiles);
  slot->epoch++;
  return slot;
}

// One band launch on `st` (heavy-first tile order for uncounted launches), then, when counting,
// the fold of the counter replicas into `cnt` (accumulating). ev_begin / ev_end: optional device
// timestamps of the kernel's start and end.
void launch(const vrt_ctx* ctx, Shard& s, vrt::KArgs a, float4* out, vrt_hit* hit, unsigned long long* cnt,
            hipStream_t st, hipEvent_t ev_begin = nullptr, hipEvent_t ev_end = nullptr, bool allow_defer = true,
            bool lone = false) {
  const bool stats = hit || cnt;
  OrderSlot* slot = stats ? nullptr : launch_state_begin(ctx, s, a, st, allow_defer || lone, lone);
  vrt::launch_render(a, stats, s.d_vox_pad, out, hit, cnt ? s.d_cnt_rep : nullptr, st, ev_begin, ev_end);
  slot_launched(s, slot, st);
  if (cnt) vrt::launch_reduce_counters(s.d_cnt_rep, cnt, st);
}

int volume_alloc(vrt_ctx* ctx, Shard& s, int32_t n) {
  if (n < 2 || n > 1024 || (n & (n - 1)) != 0)
    return fail(ctx, VRT_ERR_INVALID, "volume edge must be a power of two in [2, 1024]");
  VRT_HIP(ctx, hipSetDevice(s.device));
  // frames still in flight on the lanes read the resident volume: an upload is not a hot call
  VRT_HIP(ctx, hipDeviceSynchronize());
  // octant layout while 8 padded u16 volumes stay addressable by a 32-bit byte offset
  const bool fits = uint64_t(n + 1) * (n + 1) * (n + 1) * 2 * 8 <= (uint64_t(1) << 32);
  const int32_t octants = fits && ctx->layout_req != 1 ? 8 : 1;
  if (s.d_vox && (s.n != n || s.octants != octants)) {
    (void)hipFree(s.d_vox);
    (void)hipFree(s.d_tmp);
    (void)hipFree(s.d_vox_pad);
    s.d_vox = s.d_tmp = nullptr;
    s.d_vox_pad = nullptr;
  }
  if (!s.d_vox) {
    const size_t bytes = size_t(n) * n * n, pbytes = size_t(n + 1) * (n + 1) * (n + 1) * 2 * size_t(octants);
    if (hipMalloc(&s.d_vox, bytes) != hipSuccess ||
        hipMalloc(&s.d_tmp, (octants == 8 ? 3 : 2) * bytes) != hipSuccess ||
        hipMalloc(&s.d_vox_pad, pbytes) != hipSuccess) {
      if (s.d_vox) (void)hipFree(s.d_vox);
      if (s.d_tmp) (void)hipFree(s.d_tmp);
      if (s.d_vox_pad) (void)hipFree(s.d_vox_pad);
      s.d_vox = s.d_tmp = nullptr;
      s.d_vox_pad = nullptr;
      return fail(ctx, VRT_ERR_OOM, "hipMalloc volume buffers");
    }
  }
  s.n = n;
  s.octants = octants;
  return VRT_OK;
}

int volume_alloc_all(vrt_ctx* ctx, int32_t n) {
  for (Shard& s : ctx->sh) {
    const int st = volume_alloc(ctx, s, n);
    if (st != VRT_OK) return st;
  }
  return VRT_OK;
}

// Distance passes + packing + glass share on every device (canonical bytes already resident on
// each, ordered on part[0]), then wait (upload is not a hot call).
int volume_finish_all(vrt_ctx* ctx) {
  for (Shard& s : ctx->sh) {
    VRT_HIP(ctx, hipSetDevice(s.device));
    const uint64_t vol = uint64_t(s.n) * s.n * s.n;
    vrt::launch_volume_passes(s.d_vox, s.d_tmp, s.d_vox_pad, uint32_t(s.n), s.octants, main_stream(s));
    // certified walks cannot settle glass pixels (their secondary rays start at the exact hit
    // point) and a glass pixel pays the certified primary walk before the exact path: the
    // automatic mode turns them off when glass makes up more than 1/8 of the non-empty voxels
    if (!s.d_vstats) VRT_HIP(ctx, hipMalloc(&s.d_vstats, 2 * sizeof(unsigned long long)));
    VRT_HIP(ctx, hipMemsetAsync(s.d_vstats, 0, 2 * sizeof(unsigned long long), main_stream(s)));
    vrt::launch_glass_share(s.d_vox, vol, s.d_vstats, main_stream(s));
    VRT_HIP(ctx, hipGetLastError());
  }
  for (Shard& s : ctx->sh) {
    VRT_HIP(ctx, hipSetDevice(s.device));
    unsigned long long vs[2] = {0, 0};
    VRT_HIP(ctx, hipMemcpyAsync(vs, s.d_vstats, sizeof(vs), hipMemcpyDeviceToHost, main_stream(s)));
    VRT_HIP(ctx, hipStreamSynchronize(main_stream(s)));
    s.cert_auto = vs[0] * 8 <= vs[1];
    s.has_glass = vs[0] > 0;
  }
  ctx->err.clear();
  return VRT_OK;
}

// The first device's canonical volume (resident, ordered on its part[0]) to every other device:
// ncclBroadcast over xGMI, or device-to-device copies when a device repeats.
int broadcast_volume(vrt_ctx* ctx) {
  const size_t k = ctx->sh.size();
  if (k == 1 && !ctx->coll1) return VRT_OK;
  Shard& root = ctx->sh[0];
  const size_t bytes = size_t(root.n) * root.n * root.n;
  if (ctx->distinct) {
    VRT_NCCL(ctx, ncclGroupStart());
    for (size_t j = 0; j < k; ++j) {
      Shard& s = ctx->sh[j];
      (void)hipSetDevice(s.device);
      const ncclResult_t r = ncclBroadcast(root.d_vox, s.d_vox, bytes, ncclUint8, 0, ctx->comms[j], main_stream(s));
      if (r != ncclSuccess) {
        (void)ncclGroupEnd();
        return nccl_fail(ctx, r, "ncclBroadcast(volume)");
      }
    }
    VRT_NCCL(ctx, ncclGroupEnd());
    return VRT_OK;
  }
  VRT_HIP(ctx, hipSetDevice(root.device));
  VRT_HIP(ctx, hipEventRecord(root.ev_gs, main_stream(root)));
  for (size_t j = 1; j < k; ++j) {
    Shard& s = ctx->sh[j];
    VRT_HIP(ctx, hipSetDevice(s.device));
    VRT_HIP(ctx, hipStreamWaitEvent(main_stream(s), root.ev_gs, 0));
    VRT_HIP(ctx, hipMemcpyPeerAsync(s.d_vox, s.device, root.d_vox, root.device, bytes, main_stream(s)));
  }
  return VRT_OK;
}

// Whole-frame band buffers of every device for a W x H frame (history black on (re)creation):
// the ring of filtered bands and the ring of raw bands; with several devices, the first device's
// ring of assembled frames.
int ensure_history(vrt_ctx* ctx, int32_t w, int32_t h) {
  if (w == ctx->hist_w && h == ctx->hist_h) return VRT_OK;
  const int32_t k = int32_t(ctx->sh.size());
  const size_t pixels = size_t(band_cap(h, k)) * size_t(w);
  for (Shard& s : ctx->sh) {
    VRT_HIP(ctx, hipSetDevice(s.device));
    VRT_HIP(ctx, hipDeviceSynchronize());  // nothing may still read the old buffers
    if (pixels > s.hist_pixels) {
      for (int r = 0; r < kRing; ++r)
        for (uint32_t** b : {&s.d_ring[r], &s.d_rawbuf[r]}) {
          if (*b) (void)hipFree(*b);
          *b = nullptr;
        }
      s.hist_pixels = 0;
      for (int r = 0; r < kRing; ++r)
        for (uint32_t** b : {&s.d_ring[r], &s.d_rawbuf[r]})
          if (hipMalloc(b, pixels * 4) != hipSuccess) return fail(ctx, VRT_ERR_OOM, "hipMalloc history buffers");
      s.hist_pixels = pixels;
    }
    for (int r = 0; r < kRing; ++r) {
      VRT_HIP(ctx, hipMemset(s.d_ring[r], 0, pixels * 4));
      VRT_HIP(ctx, hipMemset(s.d_rawbuf[r], 0, pixels * 4));
      s.band_read_valid[r] = false;
    }
    for (int l = 0; l < kLanes; ++l) s.lane_parts[l] = 0;
    for (int r = 0; r < kRing; ++r) s.slot_reader[r] = 0;
  }
  if (k > 1 || ctx->coll1) {
    VRT_HIP(ctx, hipSetDevice(ctx->sh[0].device));
    for (uint32_t*& f : ctx->d_frames) {
      if (f) (void)hipFree(f);
      f = nullptr;
      if (hipMalloc(&f, size_t(w) * size_t(h) * 4) != hipSuccess) return fail(ctx, VRT_ERR_OOM, "hipMalloc frames");
    }
  }
  ctx->hist_w = w;
  ctx->hist_h = h;
  ctx->fk = 0;
  ctx->reset_pending = false;
  for (bool& v : ctx->raw_is_cur) v = false;
  for (bool& v : ctx->consumed_valid) v = false;
  for (bool& v : ctx->slot_valid) v = false;
  ctx->frame_stream = nullptr;
  return VRT_OK;
}

// st waits for every launch of lane l's last frame except the one on st itself (stream order)
int wait_lane(vrt_ctx* ctx, Shard& s, int l, hipStream_t st) {
  for (int r = 0; r < s.lane_parts[l]; ++r)
    if (s.ls[l][r] != st) VRT_HIP(ctx, hipStreamWaitEvent(st, s.ev_done[l][r], 0));
  return VRT_OK;
}

// Launch one whole frame on every device, on lane g = fk % kLanes: band j as nparts launches on
// the lane's streams — one exact-instance launch when counting or writing hit records; one launch
// when `overlap` (device-output frames, which overlap each other) and the frame does not read its
// history; else kParts interleaved parts, whose launches fill each other's tails. rgba8: the
// temporal path from the history (ring[(fk-1) % kRing], or after vrt_history_reset the last raw
// frame) into ring[fk % kRing] (+ the raw band when u_Alpha != 1: at u_Alpha = 1 the filtered
// frame is the quantised frame); else the float band into d_out (+ d_hit). Every launch records
// its lane's done event; cross-lane ordering only where buffers are shared:
//  - the lane's previous frame had another layout: its launches on the other streams (same slot);
//  - the frame reads its history (u_Alpha != 1): frame fk-1's launches (its slot, other lane);
//  - a frame read this slot as its history: its lane's last launches (WAR; that lane's later
//    frames end after it);
//  - a device-output gather of frame fk-4 read this slot: its gather stream;
//  - wait_consumed: the caller's consumption of the device-output frame in this slot.
// timing: device timestamps of every launch (vrt_stats.kernel_ms; synchronous calls only).
int launch_frame(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* p, float alpha, bool rgba8,
                 bool hits, bool counting, bool timing, bool overlap, hipEvent_t wait_consumed = nullptr,
                 bool one_part = false) {
  const int32_t k = int32_t(ctx->sh.size()), w = cam->width, h = cam->height;
  const uint64_t f = ctx->fk;
  const int g = int(f % kLanes), slot = int(f % kRing), pslot = int((f + kRing - 1) % kRing);
  // the kernel reads the history iff u_Alpha != 1 (store_pixel, vrt_render.hip)
  const bool hist = rgba8 && alpha != 1.0f;
  const bool single = counting || hits;  // one counter replica set: one counted launch
  // one_part: device-output frames consumed on their own stream (vrt_frame_stream)
  // k > 1: one launch per block-cyclic band (a band's blocks are not split into parts)
  // a synchronous whole frame that lone_defers: one launch (certified pass + exact pass)
  const bool lone = !overlap && !single && !hist && k == 1 &&
                    lone_defers(ctx, ctx->sh[0], make_args(ctx, ctx->sh[0], cam, p, 0, h, 1));
  const int nparts = single || one_part || (overlap && !hist) || lone || k > 1 ? 1 : kParts;
  for (int32_t j = 0; j < k; ++j) {
    Shard& s = ctx->sh[j];
    VRT_HIP(ctx, hipSetDevice(s.device));
    for (int q = 0; q < kParts; ++q) s.timed[q] = false;
    const int32_t hb = band_rows(h, k, j);
    if (hb == 0) {
      s.lane_parts[g] = 0;
      continue;
    }
    int st;
    for (int q = 0; q < nparts; ++q) {
      hipStream_t sq = s.ls[g][q];
      if (s.lane_parts[g] != nparts && (st = wait_lane(ctx, s, g, sq)) != VRT_OK) return st;
      if (rgba8 && f > 0) {
        const int pg = int((f - 1) % kLanes);
        if (hist) {  // part q's history rows: frame f-1's launch with the same rows, or all of them
          if (s.lane_parts[pg] == nparts) VRT_HIP(ctx, hipStreamWaitEvent(sq, s.ev_done[pg][q], 0));
          else if ((st = wait_lane(ctx, s, pg, sq)) != VRT_OK) return st;
        }
      }
      if (rgba8 && s.slot_reader[slot] > 0 && (st = wait_lane(ctx, s, s.slot_reader[slot] - 1, sq)) != VRT_OK)
        return st;
      if (rgba8 && s.band_read_valid[slot]) VRT_HIP(ctx, hipStreamWaitEvent(sq, s.ev_band_read[slot], 0));
      if (wait_consumed) VRT_HIP(ctx, hipStreamWaitEvent(sq, wait_consumed, 0));
    }
    if (rgba8) s.band_read_valid[slot] = false;
    if (counting)
      VRT_HIP(ctx, hipMemsetAsync(s.d_cnt, 0, sizeof(unsigned long long) * VRT_CNT_COUNT, s.ls[g][0]));
    const uint32_t* hsrc = ctx->reset_pending && !ctx->raw_is_cur[pslot] ? s.d_rawbuf[pslot] : s.d_ring[pslot];
    for (int q = 0; q < nparts; ++q) {
      const BandGeom bg = block_band(h, k, frame_block(k), j);
      const PartRows pr = nparts == 1 ? PartRows{bg.row0, bg.rows, bg.row_step, 0} : part_rows(h, k, kParts, j, q);
      if (pr.rows == 0) {
        VRT_HIP(ctx, hipEventRecord(s.ev_done[g][q], s.ls[g][q]));
        continue;
      }
      vrt::KArgs a = make_args(ctx, s, cam, p, pr.row0, pr.rows, pr.row_step);
      a.row_blk_sh = nparts == 1 ? bg.sh : 0;
      a.pitch = int32_t(int64_t(w) * nparts);
      const size_t off = size_t(pr.band_row0) * size_t(w);
      s.timed[q] = timing;
      hipEvent_t kb = timing ? s.ev_kbeg[q] : nullptr, ke = timing ? s.ev_kend[q] : nullptr;
      if (rgba8) {
        a.alpha = alpha;
        a.prev = hsrc + off;
        a.cur = s.d_ring[slot] + off;
        a.raw = hist ? s.d_rawbuf[slot] + off : nullptr;
        launch(ctx, s, a, nullptr, nullptr, counting ? s.d_cnt : nullptr, s.ls[g][q], kb, ke, overlap, lone);
      } else {
        launch(ctx, s, a, s.d_out + off, hits ? s.d_hit + off : nullptr, counting ? s.d_cnt : nullptr,
               s.ls[g][q], kb, ke, overlap, lone);
      }
      VRT_HIP(ctx, hipGetLastError());
      VRT_HIP(ctx, hipEventRecord(s.ev_done[g][q], s.ls[g][q]));
    }
    s.lane_parts[g] = nparts;
    if (rgba8) {
      s.slot_reader[slot] = 0;
      if (hist) s.slot_reader[pslot] = g + 1;
    }
  }
  if (rgba8) {
    ctx->raw_is_cur[slot] = !hist;
    ctx->reset_pending = false;
  }
  return VRT_OK;
}

// Wait for every device, then fill stats: kernel_ms = the slowest device's span from its first
// launch's start to its last launch's end (device timestamps: the GPU time of the frame, as
// GL_TIME_ELAPSED measured the draw); counters summed.
int finish_frame(vrt_ctx* ctx, vrt_stats* stats, bool counting) {
  float ms_max = 0.0f;
  unsigned long long tot[VRT_CNT_COUNT] = {0};
  for (Shard& s : ctx->sh) {
    VRT_HIP(ctx, hipSetDevice(s.device));
    for (int l = 0; l < kLanes; ++l)
      for (int q = 0; q < kParts; ++q) VRT_HIP(ctx, hipStreamSynchronize(s.ls[l][q]));
    VRT_HIP(ctx, hipStreamSynchronize(s.gs));
    if (stats) {
      int first = -1;
      for (int q = 0; q < kParts; ++q)
        if (s.timed[q] && first < 0) first = q;
      if (first >= 0) {  // times relative to the first launch's start (may be negative)
        float lo = 0.0f, hi = 0.0f;
        for (int q = 0; q < kParts; ++q) {
          if (!s.timed[q]) continue;
          float b = 0.0f, e = 0.0f;
          VRT_HIP(ctx, hipEventElapsedTime(&b, s.ev_kbeg[first], s.ev_kbeg[q]));
          VRT_HIP(ctx, hipEventElapsedTime(&e, s.ev_kbeg[first], s.ev_kend[q]));
          lo = std::min(lo, b);
          hi = std::max(hi, e);
        }
        ms_max = std::max(ms_max, hi - lo);
      }
    }
    if (counting) {
      unsigned long long c[VRT_CNT_COUNT];
      VRT_HIP(ctx, hipMemcpy(c, s.d_cnt, sizeof(c), hipMemcpyDeviceToHost));
      for (int q = 0; q < VRT_CNT_COUNT; ++q) tot[q] += c[q];
    }
  }
  if (stats) {
    stats->kernel_ms = ms_max;
    if (counting)
      for (int q = 0; q < VRT_CNT_COUNT; ++q) stats->counters[q] = tot[q];
  }
  return VRT_OK;
}

// Pinned host staging of synchronous frames, at least `bytes` (portable: every device's DMA
// engine writes it directly, so the k band copies run in parallel)
int ensure_stage(vrt_ctx* ctx, size_t bytes) {
  if (ctx->h_stage_bytes >= bytes) return VRT_OK;
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  ctx->h_stage = nullptr;
  ctx->h_stage_bytes = 0;
  if (hipHostMalloc(&ctx->h_stage, bytes, hipHostMallocPortable) != hipSuccess)
    return fail(ctx, VRT_ERR_OOM, "hipHostMalloc staging");
  ctx->h_stage_bytes = bytes;
  return VRT_OK;
}

// Band j's rows (band row r = frame row j + r*k) into their frame rows of the pinned staging
// buffer at byte offset stage_off: one strided DMA per device on its own link, after every launch
// of the frame on lane g. The caller copies the staged frame out after finish_frame.
int stage_bands(vrt_ctx* ctx, int g, int32_t w, int32_t h, const void* const* bands, size_t elem,
                size_t stage_off) {
  const int32_t k = int32_t(ctx->sh.size());
  for (int32_t j = 0; j < k; ++j) {
    Shard& s = ctx->sh[j];
    BandCopy bc[2];
    const int nc = band_copies(w, h, k, frame_block(k), j, elem, bc);
    if (nc == 0) continue;
    VRT_HIP(ctx, hipSetDevice(s.device));
    int st = wait_lane(ctx, s, g, s.ls[g][0]);
    if (st != VRT_OK) return st;
    for (int c = 0; c < nc; ++c)
      VRT_HIP(ctx, hipMemcpy2DAsync(static_cast<char*>(ctx->h_stage) + stage_off + bc[c].dst_off, bc[c].dst_pitch,
                                    static_cast<const char*>(bands[j]) + bc[c].src_off, bc[c].src_pitch, bc[c].width,
                                    bc[c].rows, hipMemcpyDeviceToHost, s.ls[g][0]));
  }
  return VRT_OK;
}

// Several devices (or the one-device RCCL rehearsal): frame f's bands (launched on lane g) to the
// first device — ncclGather over xGMI on every device's gather stream, or device-to-device copies
// when a device repeats — then placed into their rows of d_frames[slot] on the first device's
// gather stream (after `reuse`, the caller's consumption of that buffer, when given); ev_gathered
// marks the assembled frame.
int gather_frame(vrt_ctx* ctx, int32_t w, int32_t h, int slot, int g, hipEvent_t reuse, const uint32_t** d_frame) {
  const int32_t k = int32_t(ctx->sh.size());
  Shard& root = ctx->sh[0];
  int st;
  const int32_t cap = band_cap(h, k);
  const size_t row = size_t(w) * 4;
  const uint32_t* src[64];
  if (ctx->distinct) {  // RCCL gather of the equal-size bands to the first device over xGMI
    if (!ctx->d_gather || size_t(k) * size_t(cap) * size_t(w) > ctx->hist_pixels_gather) {
      VRT_HIP(ctx, hipDeviceSynchronize());
      if (ctx->d_gather) (void)hipFree(ctx->d_gather);
      ctx->d_gather = nullptr;
      ctx->hist_pixels_gather = 0;
      const size_t need = size_t(k) * size_t(cap) * size_t(w);
      if (hipMalloc(&ctx->d_gather, need * 4) != hipSuccess) return fail(ctx, VRT_ERR_OOM, "hipMalloc gather");
      ctx->hist_pixels_gather = need;
    }
    for (int32_t j = 0; j < k; ++j) {  // each device's gather stream after its band's launches
      Shard& s = ctx->sh[j];
      VRT_HIP(ctx, hipSetDevice(s.device));
      if ((st = wait_lane(ctx, s, g, s.gs)) != VRT_OK) return st;
    }
    VRT_NCCL(ctx, ncclGroupStart());
    for (int32_t j = 0; j < k; ++j) {
      Shard& s = ctx->sh[j];
      (void)hipSetDevice(s.device);
      const ncclResult_t r = ncclGather(s.d_ring[slot], j == 0 ? ctx->d_gather : nullptr, size_t(cap) * row,
                                        ncclUint8, 0, ctx->comms[j], s.gs);
      if (r != ncclSuccess) {
        (void)ncclGroupEnd();
        return nccl_fail(ctx, r, "ncclGather(bands)");
      }
    }
    VRT_NCCL(ctx, ncclGroupEnd());
    for (int32_t j = 0; j < k; ++j) {  // the band's next writer (frame f + kRing) waits for this
      Shard& s = ctx->sh[j];
      VRT_HIP(ctx, hipSetDevice(s.device));
      VRT_HIP(ctx, hipEventRecord(s.ev_band_read[slot], s.gs));
      s.band_read_valid[slot] = true;
    }
    for (int32_t j = 0; j < k; ++j) src[j] = ctx->d_gather + size_t(j) * cap * w;
  } else {  // a device repeats: copy the bands device to device on the first device's stream
    VRT_HIP(ctx, hipSetDevice(root.device));
    for (int32_t j = 0; j < k; ++j)
      for (int q = 0; q < ctx->sh[j].lane_parts[g]; ++q)
        VRT_HIP(ctx, hipStreamWaitEvent(root.gs, ctx->sh[j].ev_done[g][q], 0));
    for (int32_t j = 0; j < k; ++j) src[j] = ctx->sh[j].d_ring[slot];
  }
  VRT_HIP(ctx, hipSetDevice(root.device));
  if (reuse) VRT_HIP(ctx, hipStreamWaitEvent(root.gs, reuse, 0));
  uint32_t* out = ctx->d_frames[slot];
  if (ctx->distinct) {  // the gathered bands, cap rows apart, into their frame rows: one kernel
    vrt::launch_assemble_blocks(ctx->d_gather, uint64_t(cap) * uint64_t(w), k, k > 1 ? kFrameRowBlockSh : 0, w, h,
                                out, uint64_t(w), root.gs);
    VRT_HIP(ctx, hipGetLastError());
  } else {
    for (int32_t j = 0; j < k; ++j) {  // each band's blocks into their frame rows
      BandCopy bc[2];
      const int nc = band_copies(w, h, k, frame_block(k), j, 4, bc);
      for (int c = 0; c < nc; ++c)
        VRT_HIP(ctx, hipMemcpy2DAsync(reinterpret_cast<char*>(out) + bc[c].dst_off, bc[c].dst_pitch,
                                      reinterpret_cast<const char*>(src[j]) + bc[c].src_off, bc[c].src_pitch,
                                      bc[c].width, bc[c].rows, hipMemcpyDeviceToDevice, root.gs));
    }
  }
  if (!ctx->distinct)
    for (int32_t j = 0; j < k; ++j) {  // same physical device: the bands were read here
      VRT_HIP(ctx, hipEventRecord(ctx->sh[j].ev_band_read[slot], root.gs));
      ctx->sh[j].band_read_valid[slot] = true;
    }
  VRT_HIP(ctx, hipEventRecord(ctx->ev_gathered, root.gs));
  *d_frame = out;
  return VRT_OK;
}

int create(const std::vector<int>& devs, vrt_ctx** out) {
  if (!out) return VRT_ERR_INVALID;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return VRT_ERR_DEVICE;
  if (devs.empty() || devs.size() > 64) return VRT_ERR_INVALID;
  for (int d : devs)
    if (d < 0 || d >= count) return VRT_ERR_INVALID;
  DeviceGuard guard;
  vrt_ctx* c = new vrt_ctx();
  c->sh.resize(devs.size());
  for (size_t j = 0; j < devs.size(); ++j) {
    if (shard_init(c->sh[j], devs[j]) != hipSuccess) {
      vrt_destroy(c);
      return VRT_ERR_DEVICE;
    }
    for (size_t i = 0; i < j; ++i)
      if (devs[i] == devs[j]) c->distinct = false;
  }
  if (hipSetDevice(devs[0]) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_gathered, hipEventDisableTiming) != hipSuccess ||
      [&] {
        for (hipEvent_t& e : c->ev_consumed)
          if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return true;
        for (hipEvent_t& e : c->ev_slot)
          if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return true;
        return false;
      }()) {
    vrt_destroy(c);
    return VRT_ERR_DEVICE;
  }
  if (devs.size() > 1 && c->distinct) {  // one communicator per device, this process owns them all
    c->comms.resize(devs.size());
    if (ncclCommInitAll(c->comms.data(), int(devs.size()), devs.data()) != ncclSuccess) {
      c->comms.clear();
      vrt_destroy(c);
      return VRT_ERR_DEVICE;
    }
  }
  *out = c;
  return VRT_OK;
}

}  // namespace

extern "C" {

int vrt_create(uint32_t device_mask, vrt_ctx** out) {
  std::vector<int> devs;
  for (int d = 0; d < 32; ++d)
    if (device_mask & (1u << d)) devs.push_back(d);
  if (devs.empty()) {
    if (out) *out = nullptr;
    return VRT_ERR_INVALID;
  }
  return create(devs, out);
}

int vrt_create_devices(const int32_t* devices, int32_t count, vrt_ctx** out) {
  if (!devices || count < 1) {
    if (out) *out = nullptr;
    return VRT_ERR_INVALID;
  }
  return create(std::vector<int>(devices, devices + count), out);
}

void vrt_destroy(vrt_ctx* c) {
  if (!c) return;
  DeviceGuard guard;
  for (ncclComm_t cm : c->comms) (void)ncclCommDestroy(cm);
  if (!c->rank_comms.empty()) {
    (void)hipSetDevice(c->sh[0].device);
    (void)hipDeviceSynchronize();  // no gather still runs on them
    for (ncclComm_t cm : c->rank_comms) (void)ncclCommDestroy(cm);
  }
  if (!c->sh.empty()) {
    (void)hipSetDevice(c->sh[0].device);
    if (c->d_gather) (void)hipFree(c->d_gather);
    for (uint32_t* f : c->d_frames)
      if (f) (void)hipFree(f);
    for (hipEvent_t e : c->ev_consumed)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_slot)
      if (e) (void)hipEventDestroy(e);
    if (c->ev_gathered) (void)hipEventDestroy(c->ev_gathered);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (!c->lt_ev.empty()) (void)hipDeviceSynchronize();
    for (hipEvent_t e : c->lt_ev) (void)hipEventDestroy(e);
  }
  for (Shard& s : c->sh) shard_free(s);
  delete c;
}

int vrt_device_count(const vrt_ctx* ctx) { return ctx ? int(ctx->sh.size()) : VRT_ERR_INVALID; }

int vrt_device_ordinal(const vrt_ctx* ctx, int32_t i) {
  if (!ctx || i < 0 || size_t(i) >= ctx->sh.size()) return -1;
  return ctx->sh[size_t(i)].device;
}

const char* vrt_last_error(const vrt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int vrt_band_plan(int32_t height, int32_t k, int32_t parts, int32_t* out) {
  if (height < 1 || k < 1 || parts < 1 || !out) return VRT_ERR_INVALID;
  for (int32_t j = 0; j < k; ++j)
    for (int32_t p = 0; p < parts; ++p) {
      const PartRows pr = part_rows(height, k, parts, j, p);
      int32_t* o = out + (size_t(j) * parts + p) * 4;
      o[0] = pr.row0;
      o[1] = pr.rows;
      o[2] = pr.row_step;
      o[3] = pr.band_row0;
    }
  return (height + k - 1) / k;  // the largest cyclic band
}

int vrt_band_copy_plan(int32_t width, int32_t height, int32_t k, int32_t elem_bytes, int64_t* out) {
  if (width < 1 || height < 1 || k < 1 || elem_bytes < 1 || !out) return VRT_ERR_INVALID;
  for (int32_t j = 0; j < k; ++j) {
    BandCopy bc[2];
    const int nc = band_copies(width, height, k, 1, j, size_t(elem_bytes), bc);
    int64_t* o = out + size_t(j) * 5;
    o[0] = int64_t(bc[0].dst_off);
    o[1] = int64_t(bc[0].dst_pitch);
    o[2] = int64_t(bc[0].src_pitch);
    o[3] = int64_t(bc[0].width);
    o[4] = nc ? int64_t(bc[0].rows) : 0;
  }
  return k;
}

int vrt_frame_row_block(int32_t k) { return k < 1 ? VRT_ERR_INVALID : frame_block(k); }

int vrt_block_band_plan(int32_t height, int32_t k, int32_t row_block, int32_t* out) {
  if (height < 1 || k < 1 || !out || row_block < 1 || row_block > 64 || (row_block & (row_block - 1)))
    return VRT_ERR_INVALID;
  int32_t cap = 0;
  for (int32_t j = 0; j < k; ++j) {
    // k = 1: the whole frame as one band of blocks row_block apart (the same row formula)
    const BandGeom g = k == 1 ? BandGeom{0, height, row_block, 0} : block_band(height, k, row_block, j);
    out[size_t(j) * 3 + 0] = g.row0;
    out[size_t(j) * 3 + 1] = g.rows;
    out[size_t(j) * 3 + 2] = g.row_step;
    cap = std::max(cap, g.rows);
  }
  return cap;
}

int vrt_block_copy_plan(int32_t width, int32_t height, int32_t k, int32_t row_block, int32_t elem_bytes,
                        int64_t* out) {
  if (width < 1 || height < 1 || k < 1 || elem_bytes < 1 || !out || row_block < 1 || row_block > 64 ||
      (row_block & (row_block - 1)))
    return VRT_ERR_INVALID;
  int n = 0;
  for (int32_t j = 0; j < k; ++j) {
    BandCopy bc[2];
    const int nc = k == 1 ? band_copies(width, height, 1, 1, 0, size_t(elem_bytes), bc)
                          : band_copies(width, height, k, row_block, j, size_t(elem_bytes), bc);
    for (int c = 0; c < 2; ++c) {
      int64_t* o = out + (size_t(j) * 2 + c) * 7;
      const BandCopy b = c < nc ? bc[c] : BandCopy{0, 0, 0, 0, 0, 0};
      o[0] = j;
      o[1] = int64_t(b.dst_off);
      o[2] = int64_t(b.dst_pitch);
      o[3] = int64_t(b.src_off);
      o[4] = int64_t(b.src_pitch);
      o[5] = int64_t(b.width);
      o[6] = int64_t(b.rows);
      n += c < nc ? 1 : 0;
    }
  }
  return n;
}

int vrt_upload_volume(vrt_ctx* ctx, const vrt_volume* vol) {
  if (!ctx) return VRT_ERR_INVALID;
  if (!vol || !vol->voxels) return fail(ctx, VRT_ERR_INVALID, "null volume");
  DeviceGuard guard;
  int st = volume_alloc_all(ctx, vol->n);
  if (st != VRT_OK) return st;
  Shard& root = ctx->sh[0];
  const size_t bytes = size_t(vol->n) * vol->n * vol->n;
  VRT_HIP(ctx, hipSetDevice(root.device));
  VRT_HIP(ctx, hipMemcpyAsync(root.d_vox, vol->voxels, bytes, hipMemcpyHostToDevice, main_stream(root)));
  if ((st = broadcast_volume(ctx)) != VRT_OK) return st;
  return volume_finish_all(ctx);
}

int vrt_upload_volume_device(vrt_ctx* ctx, const uint8_t* d_voxels, int32_t n, void* hip_stream) {
  if (!ctx) return VRT_ERR_INVALID;
  if (!d_voxels) return fail(ctx, VRT_ERR_INVALID, "null volume");
  DeviceGuard guard;
  int st = volume_alloc_all(ctx, n);
  if (st != VRT_OK) return st;
  Shard& root = ctx->sh[0];
  const size_t bytes = size_t(n) * n * n;
  VRT_HIP(ctx, hipSetDevice(root.device));
  // ordered after the caller's work on hip_stream (which produced d_voxels)
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  VRT_HIP(ctx, hipMemcpyAsync(root.d_vox, d_voxels, bytes, hipMemcpyDeviceToDevice, s));
  VRT_HIP(ctx, hipEventRecord(root.ev_gs, s));
  VRT_HIP(ctx, hipStreamWaitEvent(main_stream(root), root.ev_gs, 0));
  if ((st = broadcast_volume(ctx)) != VRT_OK) return st;
  return volume_finish_all(ctx);
}

int vrt_build_scene_device(vrt_ctx* ctx, int32_t scene, int32_t n, uint32_t seed, void* hip_stream) {
  if (!ctx) return VRT_ERR_INVALID;
  if (scene != VRT_SCENE_TERRAIN && scene != VRT_SCENE_GLASS_CUBE && scene != VRT_SCENE_REFRACTION)
    return fail(ctx, VRT_ERR_INVALID, "unknown scene");
  if (n < 8) return fail(ctx, VRT_ERR_INVALID, "scene edge must be >= 8");
  DeviceGuard guard;
  const int st = volume_alloc_all(ctx, n);
  if (st != VRT_OK) return st;
  std::vector<float> noise;
  if (scene == VRT_SCENE_TERRAIN) {  // the heightfield (n*n floats) is built on the host
    noise.resize(size_t(n) * n);
    if (vrt_terrain_noise(n, seed, noise.data()) != VRT_OK) return fail(ctx, VRT_ERR_INVALID, "noise");
  }
  hipStream_t cs = static_cast<hipStream_t>(hip_stream);
  for (Shard& s : ctx->sh) {  // every device builds its own replica: no transfer
    VRT_HIP(ctx, hipSetDevice(s.device));
    const float* d_noise = nullptr;
    if (!noise.empty()) {
      // d_tmp (>= 2 N^3 bytes >= 4 N^2) is free until the distance passes
      VRT_HIP(ctx, hipMemcpyAsync(s.d_tmp, noise.data(), noise.size() * sizeof(float),
                                  hipMemcpyHostToDevice, main_stream(s)));
      d_noise = reinterpret_cast<const float*>(s.d_tmp);
    }
    if (&s == &ctx->sh[0] && cs) {  // ordered after the caller's prior work on its stream
      VRT_HIP(ctx, hipEventRecord(s.ev_gs, cs));
      VRT_HIP(ctx, hipStreamWaitEvent(main_stream(s), s.ev_gs, 0));
    }
    vrt::launch_build_scene(s.d_vox, scene, uint32_t(n), d_noise, main_stream(s));
    VRT_HIP(ctx, hipGetLastError());
  }
  return volume_finish_all(ctx);
}

const uint8_t* vrt_volume_device_ptr(const vrt_ctx* ctx) { return ctx ? ctx->sh[0].d_vox : nullptr; }

int vrt_debug_packed_volume(vrt_ctx* ctx, uint16_t* out, uint64_t count) {
  if (!ctx) return VRT_ERR_INVALID;
  Shard& s = ctx->sh[0];
  if (!s.d_vox_pad) return fail(ctx, VRT_ERR_NO_VOLUME, "no volume uploaded");
  const uint64_t p = uint64_t(s.n) + 1, total = p * p * p * uint64_t(s.octants);
  if (!out || count < total) return fail(ctx, VRT_ERR_INVALID, "output smaller than octants x (N+1)^3");
  DeviceGuard guard;
  VRT_HIP(ctx, hipSetDevice(s.device));
  VRT_HIP(ctx, hipMemcpy(out, s.d_vox_pad, total * sizeof(uint16_t), hipMemcpyDeviceToHost));
  return VRT_OK;
}

int vrt_set_skip_layout(vrt_ctx* ctx, int32_t octants) {
  if (!ctx) return VRT_ERR_INVALID;
  if (octants != 0 && octants != 1 && octants != 8)
    return fail(ctx, VRT_ERR_INVALID, "skip layout must be 0 (auto), 1 or 8");
  ctx->layout_req = octants;
  return VRT_OK;
}

int vrt_set_launch_timing(vrt_ctx* ctx, int32_t launches) {
  if (!ctx) return VRT_ERR_INVALID;
  if (launches < 0 || launches > (1 << 20)) return fail(ctx, VRT_ERR_INVALID, "launches must be in [0, 2^20]");
  DeviceGuard guard;
  VRT_HIP(ctx, hipSetDevice(ctx->sh[0].device));
  if (!ctx->lt_ev.empty()) VRT_HIP(ctx, hipDeviceSynchronize());  // no launch still records into them
  for (hipEvent_t e : ctx->lt_ev) (void)hipEventDestroy(e);
  ctx->lt_ev.clear();
  ctx->lt_used = 0;
  for (int32_t i = 0; i < 2 * launches; ++i) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return fail(ctx, VRT_ERR_DEVICE, "hipEventCreate (launch timing)");
    ctx->lt_ev.push_back(e);
  }
  ctx->err.clear();
  return VRT_OK;
}

int vrt_launch_timing(vrt_ctx* ctx, double* total_ms, uint64_t* launches) {
  if (!ctx || !total_ms || !launches) return VRT_ERR_INVALID;
  DeviceGuard guard;
  VRT_HIP(ctx, hipSetDevice(ctx->sh[0].device));
  double total = 0.0;
  for (size_t i = 0; i + 1 < ctx->lt_used; i += 2) {
    VRT_HIP(ctx, hipEventSynchronize(ctx->lt_ev[i + 1]));
    float ms = 0.0f;
    VRT_HIP(ctx, hipEventElapsedTime(&ms, ctx->lt_ev[i], ctx->lt_ev[i + 1]));
    total += ms;
  }
  *total_ms = total;
  *launches = ctx->lt_used / 2;
  ctx->lt_used = 0;
  ctx->err.clear();
  return VRT_OK;
}

int vrt_set_tile_order(vrt_ctx* ctx, int32_t on) {
  if (!ctx) return VRT_ERR_INVALID;
  if (on < 0 || on > 2) return fail(ctx, VRT_ERR_INVALID, "tile order must be 0, 1 or 2");
  ctx->tile_order = on;
  ctx->err.clear();
  return VRT_OK;
}

int vrt_set_exact_pass(vrt_ctx* ctx, int32_t on) {
  if (!ctx) return VRT_ERR_INVALID;
  if (on < 0 || on > 2) return fail(ctx, VRT_ERR_INVALID, "exact pass must be 0, 1 or 2");
  ctx->exact_pass = on;
  ctx->err.clear();
  return VRT_OK;
}

int vrt_set_certified(vrt_ctx* ctx, int32_t mode) {
  if (!ctx) return VRT_ERR_INVALID;
  if (mode < -1 || mode > 1) return fail(ctx, VRT_ERR_INVALID, "certified mode must be -1, 0 or 1");
  ctx->cert_req = mode;
  return VRT_OK;
}

int vrt_certified(const vrt_ctx* ctx) {
  if (!ctx) return VRT_ERR_INVALID;
  const Shard& s = ctx->sh[0];
  return s.octants == 8 && ctx->cert_req >= 0 && (ctx->cert_req > 0 || s.cert_auto || ctx->tree_req != 0) ? 1 : 0;
}

int vrt_set_cert_trees(vrt_ctx* ctx, int32_t on) {
  if (!ctx) return VRT_ERR_INVALID;
  if (on < 0 || on > 2) return fail(ctx, VRT_ERR_INVALID, "certified trees must be 0, 1 or 2");
  ctx->tree_req = on;
  ctx->err.clear();
  return VRT_OK;
}

int vrt_volume_octants(const vrt_ctx* ctx) {
  if (!ctx) return VRT_ERR_INVALID;
  return ctx->sh[0].d_vox_pad ? ctx->sh[0].octants : 0;
}

int vrt_debug_fast_math(vrt_ctx* ctx, uint64_t* out) {
  if (!ctx) return VRT_ERR_INVALID;
  if (!out) return fail(ctx, VRT_ERR_INVALID, "null output");
  DeviceGuard guard;
  VRT_HIP(ctx, hipSetDevice(ctx->sh[0].device));
  unsigned long long c[7];
  const int st = vrt::run_fast_math_check(c);
  if (st != VRT_OK) return fail(ctx, st, "vrt_debug_fast_math");
  for (int i = 0; i < 7; ++i) out[i] = c[i];
  return VRT_OK;
}

int vrt_debug_randomize(vrt_ctx* ctx, const float* dir, const float* pos, int32_t n, float randomness,
                        float seed, float* out) {
  if (!ctx) return VRT_ERR_INVALID;
  if (!dir || !pos || !out || n < 0) return fail(ctx, VRT_ERR_INVALID, "null buffer or n < 0");
  if (n == 0) return VRT_OK;
  DeviceGuard guard;
  VRT_HIP(ctx, hipSetDevice(ctx->sh[0].device));
  const size_t bytes = size_t(n) * 3 * sizeof(float);
  float *d_dir = nullptr, *d_pos = nullptr, *d_out = nullptr;
  if (hipMalloc(&d_dir, bytes) != hipSuccess || hipMalloc(&d_pos, bytes) != hipSuccess ||
      hipMalloc(&d_out, bytes) != hipSuccess) {
    (void)hipFree(d_dir);
    (void)hipFree(d_pos);
    return fail(ctx, VRT_ERR_OOM, "hipMalloc");
  }
  hipError_t e = hipMemcpy(d_dir, dir, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_pos, pos, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    vrt::launch_randomize(d_dir, d_pos, n, randomness, seed, d_out, nullptr);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, d_out, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(d_dir);
  (void)hipFree(d_pos);
  (void)hipFree(d_out);
  if (e != hipSuccess) return hip_fail(ctx, e, "vrt_debug_randomize");
  return VRT_OK;
}

// Band arguments shared by the async entry points: rows inside the image, pitch >= width; blocks
// of row_block rows (a power of two <= 64) that do not overlap (row_step >= row_block unless the
// band is one block). *sh receives log2(row_block).
static int check_band(vrt_ctx* ctx, const vrt_camera* cam, int32_t row0, int32_t rows, int32_t row_step,
                      int64_t pitch, int32_t row_block = 1, int32_t* sh = nullptr) {
  int32_t b = 0;
  while (b < 7 && (1 << b) != row_block) ++b;
  if (b == 7) return fail(ctx, VRT_ERR_INVALID, "row_block must be a power of two in [1, 64]");
  if (sh) *sh = b;
  const int64_t last = rows > 0 ? int64_t(row0) + int64_t((rows - 1) >> b) * row_step + ((rows - 1) & (row_block - 1)) : 0;
  if (rows < 0 || row_step < 1 || row0 < 0 || (rows > row_block && row_step < row_block) ||
      (rows > 0 && last >= cam->height))
    return fail(ctx, VRT_ERR_INVALID, "row band outside the image");
  if (pitch < cam->width || pitch > INT32_MAX) return fail(ctx, VRT_ERR_INVALID, "row pitch must be >= the image width");
  return VRT_OK;
}

// The next launch's timestamp events (vrt_set_launch_timing), or none when off / all in use
void launch_timing_events(vrt_ctx* ctx, hipEvent_t& begin, hipEvent_t& end) {
  begin = end = nullptr;
  if (ctx->lt_used + 2 > ctx->lt_ev.size()) return;
  begin = ctx->lt_ev[ctx->lt_used++];
  end = ctx->lt_ev[ctx->lt_used++];
}

int vrt_render_blocks_pitched_async(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* p, int32_t row0,
                                    int32_t rows, int32_t row_step, int32_t row_block, int64_t pitch,
                                    float* d_out_rgba, vrt_hit* d_out_hit, uint64_t* d_counters, void* hip_stream) {
  if (!ctx) return VRT_ERR_INVALID;
  int st = check_render_args(ctx, cam, p);
  if (st != VRT_OK) return st;
  if (!d_out_rgba) return fail(ctx, VRT_ERR_INVALID, "null output");
  int32_t sh = 0;
  if ((st = check_band(ctx, cam, row0, rows, row_step, pitch, row_block, &sh)) != VRT_OK) return st;
  if (rows == 0) return VRT_OK;
  Shard& s = ctx->sh[0];
  vrt::KArgs a = make_args(ctx, s, cam, p, row0, rows, row_step);
  a.row_blk_sh = sh;
  a.pitch = int32_t(pitch);
  hipEvent_t eb, ee;
  launch_timing_events(ctx, eb, ee);
  launch(ctx, s, a, reinterpret_cast<float4*>(d_out_rgba), d_out_hit,
         reinterpret_cast<unsigned long long*>(d_counters), static_cast<hipStream_t>(hip_stream), eb, ee);
  VRT_HIP(ctx, hipGetLastError());
  return VRT_OK;
}

int vrt_render_rows_pitched_async(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* p, int32_t row0,
                                  int32_t rows, int32_t row_step, int64_t pitch, float* d_out_rgba,
                                  vrt_hit* d_out_hit, uint64_t* d_counters, void* hip_stream) {
  return vrt_render_blocks_pitched_async(ctx, cam, p, row0, rows, row_step, 1, pitch, d_out_rgba, d_out_hit,
                                         d_counters, hip_stream);
}

int vrt_render_rows_async(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* p, int32_t row0, int32_t rows,
                          int32_t row_step, float* d_out_rgba, vrt_hit* d_out_hit, uint64_t* d_counters,
                          void* hip_stream) {
  if (!ctx) return VRT_ERR_INVALID;
  if (!cam) return fail(ctx, VRT_ERR_INVALID, "null camera");
  return vrt_render_rows_pitched_async(ctx, cam, p, row0, rows, row_step, cam->width, d_out_rgba, d_out_hit,
                                       d_counters, hip_stream);
}

int vrt_render_temporal_blocks_pitched_async(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* p,
                                             float alpha, int32_t row0, int32_t rows, int32_t row_step,
                                             int32_t row_block, int64_t pitch, const uint32_t* d_prev_rgba8,
                                             uint32_t* d_cur_rgba8, uint32_t* d_raw_rgba8, vrt_hit* d_out_hit,
                                             uint64_t* d_counters, void* hip_stream) {
  if (!ctx) return VRT_ERR_INVALID;
  int st = check_render_args(ctx, cam, p);
  if (st != VRT_OK) return st;
  if (!d_prev_rgba8 || !d_cur_rgba8) return fail(ctx, VRT_ERR_INVALID, "null history or output");
  int32_t sh = 0;
  if ((st = check_band(ctx, cam, row0, rows, row_step, pitch, row_block, &sh)) != VRT_OK) return st;
  if (rows == 0) return VRT_OK;
  Shard& s = ctx->sh[0];
  vrt::KArgs a = make_args(ctx, s, cam, p, row0, rows, row_step);
  a.row_blk_sh = sh;
  a.pitch = int32_t(pitch);
  a.alpha = alpha;
  a.prev = d_prev_rgba8;
  a.cur = d_cur_rgba8;
  a.raw = d_raw_rgba8;
  hipEvent_t eb, ee;
  launch_timing_events(ctx, eb, ee);
  launch(ctx, s, a, nullptr, d_out_hit, reinterpret_cast<unsigned long long*>(d_counters),
         static_cast<hipStream_t>(hip_stream), eb, ee);
  VRT_HIP(ctx, hipGetLastError());
  return VRT_OK;
}

// The per-launch fields of two frames' params agree (a frame batch's launch holds one copy of
// them; only the camera and u_Time are per frame)
static bool same_launch_params(const vrt_params& q, const vrt_params& r) {
  return q.sun_dir[0] == r.sun_dir[0] && q.sun_dir[1] == r.sun_dir[1] && q.sun_dir[2] == r.sun_dir[2] &&
         q.ray_noise == r.ray_noise && q.reflection_noise == r.reflection_noise &&
         q.refraction_noise == r.refraction_noise && q.max_ray_length == r.max_ray_length &&
         q.max_reflections == r.max_reflections && q.max_transparencies == r.max_transparencies &&
         q.color_only == r.color_only && q.atlas_rgba == r.atlas_rgba && q.atlas_size == r.atlas_size &&
         q.atlas_texture_size == r.atlas_texture_size;
}

// Frames [f0, f0 + nframes) of a batch whose per-launch params agree: the fewest launches that hold them
static int batch_run(vrt_ctx* ctx, int32_t nframes, const vrt_camera* cams, const vrt_params* p, int32_t row0,
                     int32_t rows, int32_t row_step, int32_t sh, int64_t pitch, uint32_t* const* d_cur_rgba8,
                     uint32_t* const* d_raw_rgba8, void* hip_stream) {
  Shard& s = ctx->sh[0];
  vrt::KArgs a = make_args(ctx, s, &cams[0], p, row0, rows, row_step);
  a.row_blk_sh = sh;
  a.pitch = int32_t(pitch);
  a.alpha = 1.0f;  // frames of a batch are independent: no history is read
  a.prev = d_cur_rgba8[0];
  a.cur = d_cur_rgba8[0];
  a.raw = d_raw_rgba8 ? d_raw_rgba8[0] : nullptr;
  a.time = p[0].time;
  for (int f = 1; f < nframes; ++f) {
    vrt::KArgs::FrameB& b = a.fb[f - 1];
    std::memcpy(b.inv_pv, cams[f].inv_pv, sizeof(b.inv_pv));
    b.time = p[f].time;
    b.cur = d_cur_rgba8[f];
    b.raw = d_raw_rgba8 ? d_raw_rgba8[f] : nullptr;
  }
  // a launch holds at most kOrderMaxTiles tiles (the tile order's and the deferred list's slot):
  // a larger batch is enqueued as the fewest consecutive launches that fit, of equal frame counts
  // (7 frames that fit 6 at a time: 4 + 3, not 6 + 1)
  const uint32_t ft = a.tiles;
  const int fit = int(std::max<uint32_t>(1u, std::min<uint32_t>(uint32_t(nframes), kOrderMaxTiles / std::max(ft, 1u))));
  const int nlaunch = (nframes + fit - 1) / fit;
  const int per = (nframes + nlaunch - 1) / nlaunch;
  const vrt::KArgs all = a;
  for (int f0 = 0; f0 < nframes; f0 += per) {
    const int nf = std::min(per, nframes - f0);
    vrt::KArgs b = all;
    if (f0 > 0) {  // frame f0 of the batch becomes the launch's frame 0
      const vrt::KArgs::FrameB& z = all.fb[f0 - 1];
      std::memcpy(b.inv_pv, z.inv_pv, sizeof(b.inv_pv));
      b.time = z.time;
      b.cur = z.cur;
      b.prev = z.cur;
      b.raw = z.raw;
      for (int f = 1; f < nf; ++f) b.fb[f - 1] = all.fb[f0 + f - 1];
    }
    b.nframes = nf;
    b.frame_tiles = ft;
    b.tiles = ft * uint32_t(nf);
    hipEvent_t eb, ee;
    launch_timing_events(ctx, eb, ee);
    launch(ctx, s, b, nullptr, nullptr, nullptr, static_cast<hipStream_t>(hip_stream), eb, ee);
    VRT_HIP(ctx, hipGetLastError());
  }
  return VRT_OK;
}

int vrt_render_temporal_batch_async(vrt_ctx* ctx, int32_t nframes, const vrt_camera* cams, const vrt_params* p,
                                    int32_t row0, int32_t rows, int32_t row_step, int32_t row_block, int64_t pitch,
                                    uint32_t* const* d_cur_rgba8, uint32_t* const* d_raw_rgba8, void* hip_stream) {
  if (!ctx) return VRT_ERR_INVALID;
  if (nframes < 1 || nframes > vrt::kMaxBatch || !cams || !p || !d_cur_rgba8)
    return fail(ctx, VRT_ERR_INVALID, "nframes must be in [1, 8] with a camera, params and an output per frame");
  for (int f = 0; f < nframes; ++f) {
    const int st = check_render_args(ctx, &cams[f], &p[f]);
    if (st != VRT_OK) return st;
    if (!d_cur_rgba8[f]) return fail(ctx, VRT_ERR_INVALID, "null output");
    if (cams[f].width != cams[0].width || cams[f].height != cams[0].height)
      return fail(ctx, VRT_ERR_INVALID, "the frames of a batch share the image size");
  }
  int32_t sh = 0;
  int st = check_band(ctx, &cams[0], row0, rows, row_step, pitch, row_block, &sh);
  if (st != VRT_OK) return st;
  if (nframes > 1 && rows >= 8192) return fail(ctx, VRT_ERR_UNSUPPORTED, "frame batches need bands of < 8192 rows");
  if (rows == 0) return VRT_OK;
  // runs of consecutive frames whose per-launch params agree share a launch (the reference's
  // day/night cycle moves u_SunDir every frame, main.cpp:346-348, 397-399: such frames take a
  // launch each, in order on the stream)
  for (int f0 = 0; f0 < nframes;) {
    int f1 = f0 + 1;
    while (f1 < nframes && same_launch_params(p[f1], p[f0])) ++f1;
    st = batch_run(ctx, f1 - f0, cams + f0, p + f0, row0, rows, row_step, sh, pitch, d_cur_rgba8 + f0,
                   d_raw_rgba8 ? d_raw_rgba8 + f0 : nullptr, hip_stream);
    if (st != VRT_OK) return st;
    f0 = f1;
  }
  return VRT_OK;
}

int vrt_render_temporal_rows_pitched_async(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* p,
                                           float alpha, int32_t row0, int32_t rows, int32_t row_step,
                                           int64_t pitch, const uint32_t* d_prev_rgba8, uint32_t* d_cur_rgba8,
                                           uint32_t* d_raw_rgba8, vrt_hit* d_out_hit, uint64_t* d_counters,
                                           void* hip_stream) {
  return vrt_render_temporal_blocks_pitched_async(ctx, cam, p, alpha, row0, rows, row_step, 1, pitch,
                                                  d_prev_rgba8, d_cur_rgba8, d_raw_rgba8, d_out_hit,
                                                  d_counters, hip_stream);
}

int vrt_render_temporal_rows_async(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* p, float alpha,
                                   int32_t row0, int32_t rows, int32_t row_step, const uint32_t* d_prev_rgba8,
                                   uint32_t* d_cur_rgba8, uint32_t* d_raw_rgba8, vrt_hit* d_out_hit,
                                   uint64_t* d_counters, void* hip_stream) {
  if (!ctx) return VRT_ERR_INVALID;
  if (!cam) return fail(ctx, VRT_ERR_INVALID, "null camera");
  return vrt_render_temporal_rows_pitched_async(ctx, cam, p, alpha, row0, rows, row_step, cam->width,
                                                d_prev_rgba8, d_cur_rgba8, d_raw_rgba8, d_out_hit, d_counters,
                                                hip_stream);
}

int vrt_render_frame(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* p, float alpha, uint8_t* out_rgba8,
                     vrt_stats* stats) {
  if (!ctx) return VRT_ERR_INVALID;
  int st = check_render_args(ctx, cam, p);
  if (st != VRT_OK) return st;
  if (!out_rgba8) return fail(ctx, VRT_ERR_INVALID, "null output");
  DeviceGuard guard;
  if ((st = ensure_history(ctx, cam->width, cam->height)) != VRT_OK) return st;
  const size_t bytes = size_t(cam->width) * size_t(cam->height) * 4;
  if ((st = ensure_stage(ctx, bytes)) != VRT_OK) return st;
  const bool counting = stats && (stats->request & VRT_STATS_COUNTERS);
  const int g = int(ctx->fk % kLanes), slot = int(ctx->fk % kRing);
  if ((st = launch_frame(ctx, cam, p, alpha, true, false, counting, stats != nullptr, false)) != VRT_OK) return st;
  std::vector<const void*> bands;
  for (Shard& s : ctx->sh) bands.push_back(s.d_ring[slot]);
  ctx->fk++;
  if ((st = stage_bands(ctx, g, cam->width, cam->height, bands.data(), 4, 0)) != VRT_OK) return st;
  if ((st = finish_frame(ctx, stats, counting)) != VRT_OK) return st;
  std::memcpy(out_rgba8, ctx->h_stage, bytes);
  ctx->err.clear();
  return VRT_OK;
}

int vrt_render_frame_device(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* p, float alpha,
                            void* hip_stream, const uint32_t** d_frame, vrt_stats* stats) {
  if (!ctx) return VRT_ERR_INVALID;
  int st = check_render_args(ctx, cam, p);
  if (st != VRT_OK) return st;
  if (!d_frame) return fail(ctx, VRT_ERR_INVALID, "null frame pointer");
  DeviceGuard guard;
  if ((st = ensure_history(ctx, cam->width, cam->height)) != VRT_OK) return st;
  const bool counting = stats && (stats->request & VRT_STATS_COUNTERS);
  const int32_t k = int32_t(ctx->sh.size()), w = cam->width, h = cam->height;
  Shard& root = ctx->sh[0];
  hipStream_t cs = static_cast<hipStream_t>(hip_stream);
  const uint64_t f = ctx->fk;
  const int slot = int(f % kRing), g = int(f % kLanes);
  VRT_HIP(ctx, hipSetDevice(root.device));
  if (!cs) {
    // no caller stream (ABI v9): the caller consumes each frame on the stream that produced it
    // (vrt_frame_stream), which renders the frame that next reuses its buffer, kRing frames later,
    // after that consumption: no ordering packet between streams. One launch per band (so that one
    // stream holds the whole frame), and the host stays at most kRing frames ahead.
    if (ctx->slot_valid[slot] && hipEventQuery(ctx->ev_slot[slot]) != hipSuccess)
      VRT_HIP(ctx, hipEventSynchronize(ctx->ev_slot[slot]));
    // a caller that switched from its own stream to NULL: the frame this slot held may still be
    // read there (its consumption was enqueued before call f - kRing + 1)
    if (f >= kRing) {
      const int rs = int((f - kRing + 1) % kRing);
      if (ctx->consumed_valid[rs]) {
        if (hipEventQuery(ctx->ev_consumed[rs]) != hipSuccess) VRT_HIP(ctx, hipEventSynchronize(ctx->ev_consumed[rs]));
        ctx->consumed_valid[rs] = false;
      }
    }
    if ((st = launch_frame(ctx, cam, p, alpha, true, false, counting, stats != nullptr, true, nullptr, true)) !=
        VRT_OK)
      return st;
    if (k == 1 && !ctx->coll1) {
      ctx->frame_stream = root.ls[g][0];
      *d_frame = root.d_ring[slot];
    } else {
      if ((st = gather_frame(ctx, w, h, slot, g, nullptr, d_frame)) != VRT_OK) return st;
      ctx->frame_stream = root.gs;
    }
    VRT_HIP(ctx, hipSetDevice(root.device));
    VRT_HIP(ctx, hipEventRecord(ctx->ev_slot[slot], ctx->frame_stream));
    ctx->slot_valid[slot] = true;
    ctx->fk++;
    if (stats && (st = finish_frame(ctx, stats, counting)) != VRT_OK) return st;
    ctx->err.clear();
    return VRT_OK;
  }
  // E_f: whatever the caller enqueued on its stream so far (its consumption of frames <= f - 1)
  VRT_HIP(ctx, hipEventRecord(ctx->ev_consumed[slot], cs));
  ctx->consumed_valid[slot] = true;
  // Frame f overwrites the buffer handed out at frame f - kRing, which the caller's work before
  // call f - kRing + 1 consumed: E_{f-kRing+1}. The host waits for it when it is not done yet
  // (the caller's stream is more than kRing - 1 frames behind): a swapchain's back-pressure, with
  // no ordering packet on the GPU. (Waiting for it on the lane's stream cost 0.016 ms per C3 frame:
  // the cross-queue wait packets stalled the lanes; profiles/r03_s14; the one-off script is in git history.)
  hipEvent_t reuse = nullptr;
  if (f >= kRing) {
    const int rs = int((f - kRing + 1) % kRing);
#if defined(VRT_DEV_NOQUERY)  // diagnostic builds: the wait on the GPU (the r03 s13 scheme) / none (unsafe)
    if (ctx->consumed_valid[rs]) reuse = ctx->ev_consumed[rs];
#elif defined(VRT_DEV_NOCONSUME)
    (void)rs;
#else
    if (ctx->consumed_valid[rs] && hipEventQuery(ctx->ev_consumed[rs]) != hipSuccess)
      VRT_HIP(ctx, hipEventSynchronize(ctx->ev_consumed[rs]));
#endif
  }
  if (k == 1 && !ctx->coll1) {
    // one device: the frame is rendered straight into the ring slot handed to the caller; up to
    // kLanes frames in flight (u_Alpha = 1: independent frames)
    if ((st = launch_frame(ctx, cam, p, alpha, true, false, counting, stats != nullptr, true, reuse)) != VRT_OK)
      return st;
#ifndef VRT_DEV_NOCSWAIT  // diagnostic builds only: the caller's stream not ordered after the frame (unsafe)
    for (int q = 0; q < root.lane_parts[g]; ++q) VRT_HIP(ctx, hipStreamWaitEvent(cs, root.ev_done[g][q], 0));
#endif
    *d_frame = root.d_ring[slot];
  } else {
    if ((st = launch_frame(ctx, cam, p, alpha, true, false, counting, stats != nullptr, true)) != VRT_OK) return st;
    if ((st = gather_frame(ctx, w, h, slot, g, reuse, d_frame)) != VRT_OK) return st;
    VRT_HIP(ctx, hipSetDevice(root.device));
    VRT_HIP(ctx, hipStreamWaitEvent(cs, ctx->ev_gathered, 0));
  }
  ctx->fk++;
  if (stats && (st = finish_frame(ctx, stats, counting)) != VRT_OK) return st;
  ctx->err.clear();
  return VRT_OK;
}

void* vrt_frame_stream(const vrt_ctx* ctx) { return ctx ? static_cast<void*>(ctx->frame_stream) : nullptr; }

int vrt_comm_unique_id(uint8_t* out, int32_t bytes) {
  static_assert(sizeof(ncclUniqueId) == VRT_COMM_ID_BYTES, "RCCL unique id size");
  if (!out || bytes < VRT_COMM_ID_BYTES) return VRT_ERR_INVALID;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return VRT_ERR_DEVICE;
  std::memcpy(out, &id, sizeof(id));
  return VRT_COMM_ID_BYTES;
}

int vrt_comm_join(vrt_ctx* ctx, const uint8_t* ids, int32_t count, int32_t nranks, int32_t rank) {
  if (!ctx) return VRT_ERR_INVALID;
  if (ctx->sh.size() != 1) return fail(ctx, VRT_ERR_INVALID, "vrt_comm_join: a one-device context per rank");
  if (!ids || count < 1 || count > 16 || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(ctx, VRT_ERR_INVALID, "vrt_comm_join: 1..16 ids, 0 <= rank < nranks");
  if (!ctx->rank_comms.empty()) return fail(ctx, VRT_ERR_INVALID, "vrt_comm_join: already joined");
  DeviceGuard guard;
  VRT_HIP(ctx, hipSetDevice(ctx->sh[0].device));
  for (int32_t i = 0; i < count; ++i) {  // every rank in the same order: each init waits for all ranks
    ncclUniqueId id;
    std::memcpy(&id, ids + size_t(i) * VRT_COMM_ID_BYTES, sizeof(id));
    ncclComm_t cm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&cm, nranks, id, rank);
    if (r != ncclSuccess) {
      for (ncclComm_t c2 : ctx->rank_comms) (void)ncclCommDestroy(c2);
      ctx->rank_comms.clear();
      return nccl_fail(ctx, r, "ncclCommInitRank");
    }
    ctx->rank_comms.push_back(cm);
  }
  ctx->rank_nranks = nranks;
  ctx->rank_id = rank;
  ctx->err.clear();
  return VRT_OK;
}

int vrt_gather_band_async(vrt_ctx* ctx, int32_t comm, const void* d_band, uint64_t bytes, void* d_gathered,
                          void* hip_stream) {
  if (!ctx) return VRT_ERR_INVALID;
  if (comm < 0 || size_t(comm) >= ctx->rank_comms.size())
    return fail(ctx, VRT_ERR_INVALID, "vrt_gather_band_async: no such communicator (vrt_comm_join)");
  if (!d_band || (ctx->rank_id == 0 && !d_gathered))
    return fail(ctx, VRT_ERR_INVALID, "vrt_gather_band_async: null band or (root) gather buffer");
  DeviceGuard guard;
  VRT_HIP(ctx, hipSetDevice(ctx->sh[0].device));
  VRT_NCCL(ctx, ncclGather(d_band, ctx->rank_id == 0 ? d_gathered : nullptr, size_t(bytes), ncclUint8, 0,
                           ctx->rank_comms[size_t(comm)], static_cast<hipStream_t>(hip_stream)));
  return VRT_OK;
}

int vrt_pack_rgb8_async(vrt_ctx* ctx, const uint32_t* d_rgba8, uint64_t pixels, uint8_t* d_rgb8, void* hip_stream) {
  if (!ctx) return VRT_ERR_INVALID;
  if (!d_rgba8 || !d_rgb8 || pixels % 4 != 0 || (reinterpret_cast<uintptr_t>(d_rgba8) & 15u) ||
      (reinterpret_cast<uintptr_t>(d_rgb8) & 3u))
    return fail(ctx, VRT_ERR_INVALID, "vrt_pack_rgb8_async: pixels % 4, 16-byte RGBA8 and 4-byte RGB8 alignment");
  DeviceGuard guard;
  VRT_HIP(ctx, hipSetDevice(ctx->sh[0].device));
  vrt::launch_pack_rgb8(d_rgba8, pixels, d_rgb8, static_cast<hipStream_t>(hip_stream));
  VRT_HIP(ctx, hipGetLastError());
  return VRT_OK;
}

int vrt_assemble_blocks_rgb8_async(vrt_ctx* ctx, const uint8_t* d_bands, int32_t k, int32_t band_rows_cap,
                                   int32_t width, int32_t height, int32_t row_block, uint32_t* d_frame,
                                   int64_t frame_pitch, void* hip_stream) {
  if (!ctx) return VRT_ERR_INVALID;
  int32_t sh = 0;
  while (sh < 7 && (1 << sh) != row_block) ++sh;
  if (sh == 7) return fail(ctx, VRT_ERR_INVALID, "row_block must be a power of two in [1, 64]");
  if (!d_bands || !d_frame || k < 1 || width < 4 || width % 4 || height < 1 || frame_pitch < width ||
      frame_pitch % 4 || (reinterpret_cast<uintptr_t>(d_frame) & 15u) || (reinterpret_cast<uintptr_t>(d_bands) & 3u))
    return fail(ctx, VRT_ERR_INVALID,
                "vrt_assemble_blocks_rgb8_async: width and pitch multiples of 4, 16-byte frame, 4-byte bands");
  if (largest_band(height, k, row_block) > band_rows_cap)
    return fail(ctx, VRT_ERR_INVALID, "vrt_assemble_blocks_rgb8_async: band_rows_cap below the largest band");
  DeviceGuard guard;
  VRT_HIP(ctx, hipSetDevice(ctx->sh[0].device));
  vrt::launch_assemble_blocks_rgb8(d_bands, uint64_t(band_rows_cap) * uint64_t(width), k, sh, width, height, d_frame,
                                   uint64_t(frame_pitch), static_cast<hipStream_t>(hip_stream));
  VRT_HIP(ctx, hipGetLastError());
  return VRT_OK;
}

int vrt_assemble_blocks_async(vrt_ctx* ctx, const uint32_t* d_bands, int32_t k, int32_t band_rows_cap,
                              int32_t width, int32_t height, int32_t row_block, uint32_t* d_frame,
                              int64_t frame_pitch, void* hip_stream) {
  if (!ctx) return VRT_ERR_INVALID;
  int32_t sh = 0;
  while (sh < 7 && (1 << sh) != row_block) ++sh;
  if (sh == 7) return fail(ctx, VRT_ERR_INVALID, "row_block must be a power of two in [1, 64]");
  if (!d_bands || !d_frame || k < 1 || width < 1 || height < 1 || frame_pitch < width)
    return fail(ctx, VRT_ERR_INVALID, "vrt_assemble_blocks_async: bad buffers or sizes");
  if (largest_band(height, k, row_block) > band_rows_cap)   // every band must fit its slice
    return fail(ctx, VRT_ERR_INVALID, "vrt_assemble_blocks_async: band_rows_cap below the largest band");
  DeviceGuard guard;
  VRT_HIP(ctx, hipSetDevice(ctx->sh[0].device));
  vrt::launch_assemble_blocks(d_bands, uint64_t(band_rows_cap) * uint64_t(width), k, sh, width, height, d_frame,
                              uint64_t(frame_pitch), static_cast<hipStream_t>(hip_stream));
  VRT_HIP(ctx, hipGetLastError());
  return VRT_OK;
}

int vrt_debug_collectives(vrt_ctx* ctx) {
  if (!ctx) return VRT_ERR_INVALID;
  if (ctx->sh.size() != 1 || !ctx->comms.empty())
    return fail(ctx, VRT_ERR_INVALID, "vrt_debug_collectives: a one-device context without communicators");
  DeviceGuard guard;
  int dev = ctx->sh[0].device;
  ncclComm_t comm = nullptr;
  VRT_NCCL(ctx, ncclCommInitAll(&comm, 1, &dev));
  ctx->comms.push_back(comm);
  ctx->coll1 = true;
  ctx->hist_w = ctx->hist_h = 0;  // the next frame allocates the assembled-frame ring
  ctx->err.clear();
  return VRT_OK;
}

int vrt_upload_atlas(vrt_ctx* ctx, const uint8_t* rgba, int32_t atlas_size) {
  if (!ctx) return VRT_ERR_INVALID;
  DeviceGuard guard;
  const int st = upload_atlas(ctx, rgba, atlas_size);
  if (st == VRT_OK) ctx->err.clear();
  return st;
}

int vrt_history_reset(vrt_ctx* ctx) {
  if (!ctx) return VRT_ERR_INVALID;
  // key F (main.cpp:417-421): std::swap(lastFrameBuffer, rayTraceFrameBuffer) — the next frame
  // filters against the last ray-traced frame. No buffer changes hands: the next frame reads its
  // history from the last frame's raw band (its filtered band when u_Alpha was 1, where the two
  // are equal), so a device-output frame the caller still holds stays untouched.
  ctx->reset_pending = ctx->fk > 0;
  ctx->err.clear();
  return VRT_OK;
}

int vrt_render(vrt_ctx* ctx, const vrt_camera* cam, const vrt_params* p, float* out_rgba, vrt_hit* out_hit,
               vrt_stats* stats) {
  if (!ctx) return VRT_ERR_INVALID;
  int st = check_render_args(ctx, cam, p);
  if (st != VRT_OK) return st;
  if (!out_rgba) return fail(ctx, VRT_ERR_INVALID, "null output");
  DeviceGuard guard;
  const int32_t k = int32_t(ctx->sh.size());
  const size_t pixels = size_t(band_cap(cam->height, k)) * size_t(cam->width);
  for (Shard& s : ctx->sh) {
    if (pixels <= s.out_pixels) continue;
    VRT_HIP(ctx, hipSetDevice(s.device));
    VRT_HIP(ctx, hipDeviceSynchronize());
    if (s.d_out) (void)hipFree(s.d_out);
    if (s.d_hit) (void)hipFree(s.d_hit);
    s.d_out = nullptr;
    s.d_hit = nullptr;
    s.out_pixels = 0;
    if (hipMalloc(&s.d_out, pixels * sizeof(float4)) != hipSuccess ||
        hipMalloc(&s.d_hit, pixels * sizeof(vrt_hit)) != hipSuccess)
      return fail(ctx, VRT_ERR_OOM, "hipMalloc frame buffers");
    s.out_pixels = pixels;
  }
  const size_t frame_px = size_t(cam->width) * size_t(cam->height);
  const size_t fbytes = frame_px * sizeof(float4), hbytes = out_hit ? frame_px * sizeof(vrt_hit) : 0;
  if ((st = ensure_stage(ctx, fbytes + hbytes)) != VRT_OK) return st;
  const bool counting = stats && (stats->request & VRT_STATS_COUNTERS);
  const int g = int(ctx->fk % kLanes);
  if ((st = launch_frame(ctx, cam, p, 1.0f, false, out_hit != nullptr, counting, stats != nullptr, false)) != VRT_OK)
    return st;
  std::vector<const void*> bands, hbands;
  for (Shard& s : ctx->sh) {
    bands.push_back(s.d_out);
    hbands.push_back(s.d_hit);
  }
  if ((st = stage_bands(ctx, g, cam->width, cam->height, bands.data(), sizeof(float4), 0)) != VRT_OK) return st;
  if (out_hit && (st = stage_bands(ctx, g, cam->width, cam->height, hbands.data(), sizeof(vrt_hit), fbytes)) != VRT_OK)
    return st;
  if ((st = finish_frame(ctx, stats, counting)) != VRT_OK) return st;
  std::memcpy(out_rgba, ctx->h_stage, fbytes);
  if (out_hit) std::memcpy(out_hit, static_cast<const char*>(ctx->h_stage) + fbytes, hbytes);
  ctx->err.clear();
  return VRT_OK;
}

}  // extern "C"
