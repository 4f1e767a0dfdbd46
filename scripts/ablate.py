#!/usr/bin/env python3
"""Build ablation variants of the kernel for scripts/ab.py (timing breakdown only; they render
WRONG images and are never the product library): each variant is the product source with one
text substitution, compiled into build/variants/libvrt_<name>.so.
Usage: python scripts/ablate.py [names...]   (default: all)"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "voxelraytracer_amd", "csrc")
K = "vrt_render.hip"

ABLATIONS = {
    # the sky colour: no pow / normalize, a constant sky
    "nosky": ("__device__ __forceinline__ void apply_sky_color(const Ctx& c, const Ray& ray, f3& color) {\n",
              "__device__ __forceinline__ void apply_sky_color(const Ctx& c, const Ray& ray, f3& color) {\n"
              "  color = mk(0.1f, 0.2f, 0.3f); return;\n"),
    # the lit brightness of hits: no pow / reflect
    "nolit": ("__device__ __forceinline__ float lit_brightness(const Hit& h, const f3 sun_dir, const f3 ray_dir) {\n",
              "__device__ __forceinline__ float lit_brightness(const Hit& h, const f3 sun_dir, const f3 ray_dir) {\n"
              "  return 0.7f;\n"),
    # the temporal epilogue: store the quantised colour only (no history read, no blend)
    "noepi": ("    a.cur[o] = temporal_blend(rw, a.prev[o], a.alpha);\n", "    a.cur[o] = rw;\n"),
    # certified shadow walks of certified hits: always lit
    "noshadow": ("    const CertResult s = cert_walk<true>(c, hh.point, S, c.sun_rcp, c.max_len - hh.len, ax, ay, az,\n"
                 "                                         h.eu, ed, hh.len, 0u);\n",
                 "    CertResult s; s.res = CERT_MISS;\n"),
    # the primary certified walk: every pixel a certified miss (sky), no exact path
    "nowalk": ("  CertResult h = cert_walk<false>(c, P, D, rcp, c.max_len - ray0.len, cx, cy, cz, 0.0f,\n"
               "                                  mk(0.0f, 0.0f, 0.0f), 0.0f, 0u);\n",
               "  CertResult h; h.res = CERT_MISS;\n"),
    # the exact path of unsure and glass pixels: skipped (their colour stays black)
    "noexact": ("    const bool need_exact = CERT < 2 || !cert_pixel(c, ray, color);\n",
                "    const bool need_exact = CERT < 2 || (!cert_pixel(c, ray, color) && ray.len < 0.0f);\n"),
    # the bounce stacks of glass pixels: no secondary rays
    # shadow starts the certified walk cannot place: assume lit instead of the exact path
    "nostartunsure": ("      CERT_DIAG(6);\n      return false;\n",
                      "      CERT_DIAG(6);\n      apply_hit_color<false>(c, hh, ray.energy, lit, color);\n      return true;\n"),
    # primary walks that end unsure: treat as a miss (sky) instead of the exact path
    "noprimunsure": ("  if (h.res == CERT_UNSURE) { CERT_DIAG(1); return false; }\n",
                     "  if (h.res == CERT_UNSURE) { CERT_DIAG(1); h.res = CERT_MISS; }\n"),
    # waves raise their priority when a lane enters the exact path (timing A/B, images unchanged)
    "exprio2": ("      heavy = true;\n", "      heavy = true;\n      __builtin_amdgcn_s_setprio(2);\n"),
    "exprio3": ("      heavy = true;\n", "      heavy = true;\n      __builtin_amdgcn_s_setprio(3);\n"),
    "exprio1": ("      heavy = true;\n", "      heavy = true;\n      __builtin_amdgcn_s_setprio(1);\n"),
    "nostack": ("  if (h0.found && mat_id(h0.voxel) == 2) {  // only glass spawns secondary rays (:440-448)\n",
                "  if (h0.found && mat_id(h0.voxel) == 2 && ray.len < 0.0f) {\n"),
}


# context experiments (timing only; unsafe orderings): file, anchor, replacement
CONTEXT = {
    # device-output frames: no wait for the caller's consumption of a reused ring slot
    "noconsumed": ("vrt_context.cpp", "  hipEvent_t reuse = ctx->consumed_valid[slot] ? ctx->ev_consumed[slot] : nullptr;\n",
                   "  hipEvent_t reuse = nullptr;\n"),
    # tile order for every certified-pixel launch (also volumes without glass)
    "orderall": ("vrt_context.cpp", "      !s.has_glass)", "      false)"),
}
# multi-file experiments: name -> [(file, anchor, replacement), ...]
MULTI = {
    # tile order: the second pass in reverse row order (top of the frame first)
    "pass2rev": [("vrt_render.hip", "  const uint32_t t = L - cap;\n", "  const uint32_t t = a.tiles - 1u - (L - cap);\n")],
    # bounce stacks without raised wave priority / at priority 1
    "noprio": [("vrt_render.hip", "    __builtin_amdgcn_s_setprio(kStackPrio);  // bounce stacks: the longest waves of a frame\n", "")],
    "prio1": [("vrt_render.hip", "constexpr int kStackPrio = 3;", "constexpr int kStackPrio = 1;")],
    # tile order: a tile counts as heavy only if both of its waves had exact-path pixels
    "heavy2": [("vrt_render.hip", "  if (((old + add) & 0xFF00u) != 0u) {\n", "  if (((old + add) & 0xFF00u) >= 0x200u) {\n")],
    # the tile order also for certified-exact-path launches (CERT 1: glass-heavy volumes, C1)
    "ordcert1": [
        ("vrt_context.cpp", "a.textured || a.cert != 2 ||", "a.textured || a.cert < 1 ||"),
        ("vrt_render.hip", "                                     : a.cert == 1 ? render_kernel<false, false, 1>",
         "                                     : a.cert == 1 ? (a.order ? render_kernel<false, false, 1, true> : render_kernel<false, false, 1>)"),
    ],
    # the tile-order bookkeeping out of line (codegen of the render body independent of it)
    "ordnoinline": [
        ("vrt_render.hip", "__device__ __forceinline__ uint32_t ordered_tile(", "__device__ __noinline__ uint32_t ordered_tile("),
        ("vrt_render.hip", "__device__ __forceinline__ void order_record(", "__device__ __noinline__ void order_record("),
    ],
    # heavy tiles = tiles with any exact-path pixel (not only bounce stacks), tile order on for
    # every certified-pixel launch (also without glass)
    "heavyexact": [
        ("vrt_render.hip", "      stack = exact_pixel<STATS, TEX, CERT >= 1, CERT == 2>(",
         "      stack = true; exact_pixel<STATS, TEX, CERT >= 1, CERT == 2>("),
        ("vrt_context.cpp", "      !s.has_glass)", "      false)"),
    ],
    # the same marking, tile order still only for volumes with glass
    "heavyexact2": [
        ("vrt_render.hip", "      stack = exact_pixel<STATS, TEX, CERT >= 1, CERT == 2>(",
         "      stack = true; exact_pixel<STATS, TEX, CERT >= 1, CERT == 2>("),
    ],
}


def build(name):
    if name in MULTI:
        subs = MULTI[name]
    elif name in CONTEXT:
        subs = [CONTEXT[name]]
    else:
        subs = [(K,) + ABLATIONS[name]]
    out = os.path.join(ROOT, "build", "ablate", name)
    os.makedirs(out, exist_ok=True)
    for src in os.listdir(SRC):
        shutil.copy(os.path.join(SRC, src), out)
    for f, old, new in subs:
        text = open(os.path.join(out, f)).read()
        assert text.count(old) == 1, f"{name}: anchor not found once in {f}"
        open(os.path.join(out, f), "w").write(text.replace(old, new))
    srcs = [os.path.join(out, x) for x in ("vrt_render.hip", "vrt_context.cpp", "vrt_host.cpp")]
    os.makedirs(os.path.join(ROOT, "build", "variants"), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
           "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize", "-I" + os.path.join(ROOT, "include"),
           "-I" + out, "-DVRT_DIAGNOSTIC_BUILD", "-shared", "-o",
           os.path.join(ROOT, "build", "variants", f"libvrt_{name}.so")] + srcs + \
          ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.check_call(cmd)
    print("built", name)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(ABLATIONS):
        build(n)
