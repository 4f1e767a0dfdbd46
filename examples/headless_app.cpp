// Headless AppScene: the frame loop of src/main.cpp (AppScene, :138-430) driven through the C-ABI
// of include/vrt.h instead of GL + Greet (the drop-in demonstrated in the
// reference's own language). What it mirrors:
//   - volume: the _TERRAIN / _GLASS_CUBE / _REFRACTION builders (main.cpp:218-288) ->
//     vrt_build_scene, uploaded once (replaces glTexImage3D, :315-318)
//   - camera: Perspective(aspect, 90, 0.01, 100) at the "C" key pose (-3.45, 2.17, 3.53),
//     (-33, -48, 0) degrees (:161, :171-172, :415-416) -> vrt_camera_make
//   - per frame (Render, :323-361): u_Time = 1, 2, 3, ... (:343-345), u_SunDir from timeOfDay
//     (:346-348, "Make day" = 0.9 * dayTime, :577) advanced by Update's day/night clock
//     (:397-404) when --day-night is given, noise uniforms (:156-158)
//   - RGB8 store + temporal filter + FBO swap (:363-393) -> vrt_render_frame
//   - "Clear framebuffer" (key F, :417-421) -> vrt_history_reset, via --reset-at K
//   - the GUI's FPS label from GL_TIME_ELAPSED (:350-360) -> vrt_stats.kernel_ms (timing only:
//     the fast kernel instance; --counters also counts rays, which runs the exact instance)
//   - more than one GPU (--device-mask): vrt_create's mask, the frame split into row bands
//   - --pipelined: the display path. Frames stay on the device (vrt_render_frame_device, where a
//     texture upload for display would consume them) with no per-frame host sync, so consecutive
//     frames overlap on the GPU; GPU time per frame = hipEvents around the timed frames / count.
//     The default synchronous loop waits for every frame like the reference's blocking
//     GL_TIME_ELAPSED readback (main.cpp:352-356) and reports each frame's own GPU time.
//   - Utils::Screenshot of the last frame (key F1, :424-428) -> a binary PPM (--ppm), and the raw
//     RGBA8 frame (--raw, row 0 = bottom) for tests
// Build: make app (-> build/vrt_headless). Usage: build/vrt_headless --help
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "vrt.h"

namespace {

struct Options {
  std::string scene = "refraction";
  int n = 128, width = 1920, height = 1080, frames = 10;
  int max_reflections = 4, max_transparencies = 4;
  float alpha = 1.0f, ray_noise = 0.0f, reflection_noise = 0.0f, refraction_noise = 0.0f;
  float frame_seconds = 0.0f;  // > 0: Update(timeElapsed) per frame (day/night cycle)
  int reset_at = -1;           // frame index before which key F is pressed
  std::string atlas_raw;       // textured mode: raw RGBA8 atlas file (size^2 * 4 bytes)
  int atlas_size = 256, atlas_tile = 128;
  std::string ppm, raw;
  bool quiet = false, counters = false, pipelined = false, caller_stream = false;
  uint32_t device_mask = 1;  // bit i = HIP device i
  int warmup = 0;            // frames excluded from the reported mean
};

void usage() {
  std::puts(
      "vrt_headless [--scene terrain|glass_cube|refraction] [--n N] [--size WxH] [--frames K]\n"
      "             [--bounces R T] [--alpha A] [--ray-noise x] [--reflection-noise x]\n"
      "             [--refraction-noise x] [--day-night SECONDS_PER_FRAME] [--reset-at K]\n"
      "             [--atlas-raw FILE --atlas-size S --atlas-tile T] [--ppm FILE] [--raw FILE]\n"
      "             [--device-mask M] [--counters] [--warmup K] [--pipelined [--caller-stream]] [--quiet]");
}

bool parse(int argc, char** argv, Options& o) {
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&](const char* what) -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", what);
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--scene") o.scene = next("--scene");
    else if (a == "--n") o.n = std::atoi(next("--n"));
    else if (a == "--size") {
      if (std::sscanf(next("--size"), "%dx%d", &o.width, &o.height) != 2) return false;
    } else if (a == "--frames") o.frames = std::atoi(next("--frames"));
    else if (a == "--bounces") {
      o.max_reflections = std::atoi(next("--bounces"));
      o.max_transparencies = std::atoi(next("--bounces"));
    } else if (a == "--alpha") o.alpha = std::strtof(next("--alpha"), nullptr);
    else if (a == "--ray-noise") o.ray_noise = std::strtof(next("--ray-noise"), nullptr);
    else if (a == "--reflection-noise") o.reflection_noise = std::strtof(next(a.c_str()), nullptr);
    else if (a == "--refraction-noise") o.refraction_noise = std::strtof(next(a.c_str()), nullptr);
    else if (a == "--day-night") o.frame_seconds = std::strtof(next("--day-night"), nullptr);
    else if (a == "--reset-at") o.reset_at = std::atoi(next("--reset-at"));
    else if (a == "--atlas-raw") o.atlas_raw = next("--atlas-raw");
    else if (a == "--atlas-size") o.atlas_size = std::atoi(next("--atlas-size"));
    else if (a == "--atlas-tile") o.atlas_tile = std::atoi(next("--atlas-tile"));
    else if (a == "--ppm") o.ppm = next("--ppm");
    else if (a == "--raw") o.raw = next("--raw");
    else if (a == "--quiet") o.quiet = true;
    else if (a == "--counters") o.counters = true;
    else if (a == "--pipelined") o.pipelined = true;
    else if (a == "--caller-stream") o.caller_stream = true;
    else if (a == "--device-mask") o.device_mask = uint32_t(std::strtoul(next(a.c_str()), nullptr, 0));
    else if (a == "--warmup") o.warmup = std::atoi(next("--warmup"));
    else if (a == "--help" || a == "-h") return false;
    else {
      std::fprintf(stderr, "unknown option %s\n", a.c_str());
      return false;
    }
  }
  return true;
}

int scene_id(const std::string& s) {
  if (s == "terrain") return VRT_SCENE_TERRAIN;
  if (s == "glass_cube") return VRT_SCENE_GLASS_CUBE;
  if (s == "refraction") return VRT_SCENE_REFRACTION;
  return -1;
}

bool write_file(const std::string& path, const void* data, size_t bytes) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  const bool ok = std::fwrite(data, 1, bytes, f) == bytes;
  return std::fclose(f) == 0 && ok;
}

// Utils::Screenshot equivalent: RGB, top row first (the frame's row 0 is the bottom)
bool write_ppm(const std::string& path, const std::vector<uint8_t>& rgba, int w, int h) {
  std::string img = "P6\n" + std::to_string(w) + " " + std::to_string(h) + "\n255\n";
  const size_t head = img.size();
  img.resize(head + size_t(w) * h * 3);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x)
      std::memcpy(&img[head + (size_t(h - 1 - y) * w + x) * 3], &rgba[(size_t(y) * w + x) * 4], 3);
  return write_file(path, img.data(), img.size());
}

}  // namespace

int main(int argc, char** argv) {
  // A context runs frames on up to nine streams per GPU (four lanes of frames in flight, their
  // second parts, the gather stream) beside the caller's: with HIP's default of 4 hardware queues
  // the caller's stream shares a queue with a lane and its per-frame waits stall that lane's next
  // frame (C3 0.071 vs 0.061 ms per frame). Set before the first HIP call.
  // (bench.py keeps HIP's 4: it enqueues its frames on its own four lane streams with no caller
  // stream waiting on them, one stream per queue, and 4 queues is fastest for that shape — DESIGN
  // §6 "Frames in flight"; this app's shape is vrt_render_frame_device's, a different topology.)
  setenv("GPU_MAX_HW_QUEUES", "16", 0);
  Options o;
  if (!parse(argc, argv, o)) {
    usage();
    return 2;
  }
  const int sid = scene_id(o.scene);
  if (sid < 0 || o.frames < 1) {
    usage();
    return 2;
  }
  std::vector<uint8_t> vox(size_t(o.n) * o.n * o.n);
  if (vrt_build_scene(sid, o.n, 0, vox.data()) != VRT_OK) {
    std::fprintf(stderr, "vrt_build_scene failed\n");
    return 1;
  }
  vrt_ctx* rt = nullptr;
  if (vrt_create(o.device_mask, &rt) != VRT_OK) {
    std::fprintf(stderr, "vrt_create failed: %s\n", vrt_last_error(rt));
    return 1;
  }
  int status = 0;
  const vrt_volume vol{vox.data(), o.n};
  if (vrt_upload_volume(rt, &vol) != VRT_OK) {
    std::fprintf(stderr, "vrt_upload_volume: %s\n", vrt_last_error(rt));
    vrt_destroy(rt);
    return 1;
  }
  const float pos[3] = {-3.45f, 2.17f, 3.53f}, rot[3] = {-33.0f, -48.0f, 0.0f};
  vrt_camera cam;
  vrt_camera_make(pos, rot, o.width, o.height, 90.0f, 0.01f, 100.0f, &cam);
  vrt_params p;
  vrt_params_default(&p);
  p.max_reflections = o.max_reflections;
  p.max_transparencies = o.max_transparencies;
  p.ray_noise = o.ray_noise;
  p.reflection_noise = o.reflection_noise;
  p.refraction_noise = o.refraction_noise;
  std::vector<uint8_t> atlas;
  if (!o.atlas_raw.empty()) {  // textured mode (the reference's default build)
    atlas.resize(size_t(o.atlas_size) * o.atlas_size * 4);
    FILE* f = std::fopen(o.atlas_raw.c_str(), "rb");
    if (!f || std::fread(atlas.data(), 1, atlas.size(), f) != atlas.size()) {
      std::fprintf(stderr, "cannot read %zu atlas bytes from %s\n", atlas.size(), o.atlas_raw.c_str());
      if (f) std::fclose(f);
      vrt_destroy(rt);
      return 1;
    }
    std::fclose(f);
    p.color_only = 0;
    p.atlas_rgba = atlas.data();
    p.atlas_size = o.atlas_size;
    p.atlas_texture_size = o.atlas_tile;
  }
  const float day_time = 50.0f;        // dayTime (main.cpp:153)
  float time_of_day = 0.9f * day_time;  // "Make day" (main.cpp:577)
  std::vector<uint8_t> frame(size_t(o.width) * o.height * 4);
  if (o.pipelined) {  // display path: device frames, no per-frame host sync
    // Default: no caller stream (ABI v9) — each frame is consumed on the stream that produced it
    // (vrt_frame_stream), the display path with no ordering packet between streams; time per
    // frame = wall time of the timed frames between two device synchronisations (GPU-bound).
    // --caller-stream: the frames are ordered on this host's own stream instead (each frame makes
    // it wait), timed with hipEvents on it.
    const uint32_t* d_frame = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipSetDevice(vrt_device_ordinal(rt, 0)) != hipSuccess || hipStreamCreate(&s) != hipSuccess ||
        hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
      std::fprintf(stderr, "HIP setup failed\n");
      vrt_destroy(rt);
      return 1;
    }
    hipStream_t cs = o.caller_stream ? s : nullptr;
    auto t0 = std::chrono::steady_clock::now();
    for (int f = 0; f < o.frames && status == 0; ++f) {
      if (f == o.warmup) {
        if (cs) {
          (void)hipEventRecord(e0, s);
        } else {
          if (hipDeviceSynchronize() != hipSuccess) status = 1;
          t0 = std::chrono::steady_clock::now();
        }
      }
      if (f == o.reset_at) vrt_history_reset(rt);
      p.time = float(f + 1);
      vrt_sun_dir(time_of_day, day_time, p.sun_dir);
      if (vrt_render_frame_device(rt, &cam, &p, o.alpha, cs, &d_frame, nullptr) != VRT_OK) {
        std::fprintf(stderr, "vrt_render_frame_device: %s\n", vrt_last_error(rt));
        status = 1;
      }
      if (o.frame_seconds > 0.0f) {
        time_of_day += o.frame_seconds;
        while (time_of_day > day_time) time_of_day -= day_time;
      }
    }
    float ms = 0.0f;
    if (cs) {
      (void)hipEventRecord(e1, s);
    } else if (status == 0) {
      if (hipDeviceSynchronize() != hipSuccess) status = 1;
      ms = float(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    // the last frame to the host on the stream it is consumed on
    hipStream_t consume = cs ? cs : static_cast<hipStream_t>(vrt_frame_stream(rt));
    if (status == 0 && hipMemcpyAsync(frame.data(), d_frame, frame.size(), hipMemcpyDeviceToHost, consume) != hipSuccess)
      status = 1;
    if (hipStreamSynchronize(consume) != hipSuccess) status = 1;
    if (cs) (void)hipEventElapsedTime(&ms, e0, e1);
    const int timed = o.frames - o.warmup;
    if (status == 0 && timed > 0)
      std::printf("pipelined (%s): timed %d frames (after %d warm-up) on %d device(s): mean %.4f ms per frame\n",
                  cs ? "caller stream, GPU time" : "frame streams, wall time", timed, o.warmup,
                  vrt_device_count(rt), ms / timed);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
    if (status == 0 && !o.raw.empty() && !write_file(o.raw, frame.data(), frame.size())) status = 1;
    if (status == 0 && !o.ppm.empty() && !write_ppm(o.ppm, frame, o.width, o.height)) status = 1;
    vrt_destroy(rt);
    return status;
  }
  double ms_sum = 0.0;
  int timed = 0;
  for (int f = 0; f < o.frames && status == 0; ++f) {
    if (f == o.reset_at) vrt_history_reset(rt);  // key F
    p.time = float(f + 1);                       // static i; i++ (main.cpp:343-345)
    vrt_sun_dir(time_of_day, day_time, p.sun_dir);
    vrt_stats st;
    std::memset(&st, 0, sizeof(st));
    st.request = o.counters ? VRT_STATS_COUNTERS : 0u;
    if (vrt_render_frame(rt, &cam, &p, o.alpha, frame.data(), &st) != VRT_OK) {
      std::fprintf(stderr, "vrt_render_frame: %s\n", vrt_last_error(rt));
      status = 1;
      break;
    }
    if (f >= o.warmup) {
      ms_sum += st.kernel_ms;
      ++timed;
    }
    const uint64_t rays = st.counters[VRT_CNT_PRIMARY_RAYS] + st.counters[VRT_CNT_SECONDARY_RAYS] +
                          st.counters[VRT_CNT_SHADOW_RAYS];
    if (!o.quiet && o.counters)
      std::printf("frame %d  %.4f ms  fps %.0f  rays %llu  %.0f Mrays/s\n", f, st.kernel_ms,
                  1000.0 / st.kernel_ms, (unsigned long long)rays, rays / (st.kernel_ms * 1e3));
    else if (!o.quiet)
      std::printf("frame %d  %.4f ms  fps %.0f\n", f, st.kernel_ms, 1000.0 / st.kernel_ms);
    if (o.frame_seconds > 0.0f) {  // Update(): day/night cycle (main.cpp:397-404)
      time_of_day += o.frame_seconds;
      while (time_of_day > day_time) time_of_day -= day_time;
    }
  }
  if (status == 0 && timed > 0)
    std::printf("timed %d frames (after %d warm-up) on %d device(s): mean %.4f ms GPU time per frame%s\n",
                timed, o.warmup, vrt_device_count(rt), ms_sum / timed,
                o.counters ? " (exact instance, counting)" : "");
  if (status == 0 && !o.raw.empty() && !write_file(o.raw, frame.data(), frame.size())) status = 1;
  if (status == 0 && !o.ppm.empty() && !write_ppm(o.ppm, frame, o.width, o.height)) status = 1;
  vrt_destroy(rt);
  return status;
}
