#!/usr/bin/env python3
"""Headline benchmark: Mrays/s + achieved algorithmic GB/s of the voxel ray-trace pass.

Workload (BASELINE.json metric "1920x1080 @ 128^3 voxels, 4 bounces"): configs[3], the
_REFRACTION scene at 128^3, 1920x1080, reflect+refract 4 bounces (MAX_REFLECTIONS =
MAX_TRANSPARENCIES = 4), colour-only, noise 0, camera/sun of SURVEY.md §8d. A step = one frame.

Output (default --output rgba8): the reference's stored frame, i.e. the colour written to the RGB8
ray-trace FBO and the temporal filter into the RGB8 history (main.cpp:363-393), fused into the
kernel epilogue (4 B history read + 4 B write per pixel); --output f32 writes vrt_render's float
RGBA frame (16 B per pixel).

Frames in flight: at u_Alpha = 1 (the slider default) a frame does not read its history, so
consecutive frames are independent; the timed frames rotate over --lanes (default 4) lanes, each
with its own HIP stream and output buffer, so up to four frames are in flight and the next frames'
waves fill the wave slots one frame's longest (exact-path) waves hold (voxelraytracer_amd/tiles.py;
profiles/r03_pipe). At u_Alpha != 1 frames depend on their history: one lane, two
interleaved row parts on two streams, filtered in place (the round-2 scheme).

Multi-GPU (one process per GPU, torchrun): voxelraytracer_amd/tiles.py splits the frame into
block-cyclic bands of 16 rows (rank r owns row blocks r, r+N, ...); every rank renders and filters
its band in HBM, and every timed frame is gathered to rank 0 over RCCL (xGMI) and assembled there
(north_star's "RCCL gather of per-tile RGBA"; the reference displays every frame from one device,
main.cpp:379-385): per frame, on the frame's lane stream, the render, the library's ncclGather
(one communicator per lane, vrt_gather_band_async) and rank 0's assembly kernel
(vrt_assemble_blocks_async), so the gathers of frames in flight overlap the renders of the others.
From N = 4 rank 0 is a compositor (--compositor): it renders no band and assembles every frame,
while ranks 1..N-1 split the frame (tiles.split_band_spec). A K-way band renders K frames per
launch (8 from K = 7; vrt_render_temporal_batch_async).
The JSON's "render_only" object times the same frames without the gather (labelled; --no-gather
makes that the timed path and gathers the last frame once instead). Default --scaling strong: the
config's frame (C3: 1920x1080) is split N ways, the reference's one frame per draw
(main.cpp:325-361) tiled across the GPUs; --scaling weak renders an N-fold taller frame of the same
view instead (each rank a config-sized band; opt-in, no BASELINE config names that frame).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C1|C2|C3|C4]
                       [--output rgba8|f32] [--alpha A] [--scaling strong|weak] [--lanes L]
"""
import argparse
import faulthandler
import json
import os
import signal
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# HIP spreads streams round-robin over GPU_MAX_HW_QUEUES hardware queues (HIP's default 4, and what
# the GPU box exports): the four lanes (frames in flight) then have a queue each. More queues or
# lanes are slower (C3 ms/frame at 4 / 8 / 16 queues: 4 lanes 0.0386 / 0.0388 / 0.0387, 6 lanes
# 0.0469 / 0.0435 / 0.0628, 8 lanes 0.0387 / 0.0420 / 0.0497; profiles/r03_s48). Set before HIP
# initialises, only when the environment has no value.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "4")

CONFIGS = {
    # name: (scene, N, W, H, R, T, description)
    "C0": ("glass_cube", 16, 400, 400, 1, 2, "_GLASS_CUBE 16^3 400x400 (R,T)=(1,2)"),
    "C1": ("glass_cube", 128, 1920, 1080, 1, 2, "_GLASS_CUBE 128^3 1920x1080 1 reflection (R,T)=(1,2)"),
    "C2": ("terrain", 128, 1920, 1080, 4, 2, "_TERRAIN 128^3 1920x1080 4 reflection bounces (R,T)=(4,2)"),
    "C3": ("refraction", 128, 1920, 1080, 4, 4,
           "_REFRACTION 128^3 1920x1080 reflect+refract 4 bounces (R,T)=(4,4)"),
    "C4": ("terrain", 512, 3840, 2160, 4, 2, "_TERRAIN 512^3 3840x2160 4 bounces (R,T)=(4,2)"),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS))
    ap.add_argument("--device-warmup-ms", type=float, default=200.0,
                    help="untimed frames for this long before the W warmup frames: the engine "
                         "clock's DPM ramp under this load (~1.9 -> ~2.3 GHz over the first "
                         "~150 ms, profiles/r03_s2) would otherwise be inside short timed runs")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="budget of the oracle CPU baseline sample (0 disables)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline (0: all the host grants, see host_cores)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the post-timing check of the timed frame against the exact instance")
    ap.add_argument("--verify-frames", type=int, default=1,
                    help="consecutive frames of the timed path checked after the timed region")
    ap.add_argument("--oracle-check", action="store_true",
                    help="also check the verified frames against the oracle when the CPU baseline "
                         "leg is off (renders one oracle frame on the host cores)")
    ap.add_argument("--output", default="rgba8", choices=["rgba8", "f32"],
                    help="rgba8: the reference's stored frame (RGB8 store + temporal filter fused "
                         "into the kernel); f32: the float RGBA frame of vrt_render")
    ap.add_argument("--alpha", type=float, default=1.0,
                    help="temporal filter u_Alpha (slider default 1.0, res/guis/header.xml:20)")
    ap.add_argument("--shading", default="color", choices=["color", "textured"],
                    help="color: _COLOR_ONLY materials (SURVEY §8d configs); textured: the "
                         "reference's default build, atlas shading (synthetic 256/128 atlas)")
    ap.add_argument("--atlas", default="ref", choices=["ref", "synthetic"],
                    help="textured atlas: the reference's own textures (tests/golden/atlas fixture) "
                         "or the synthetic one (fractional glass alpha)")
    ap.add_argument("--lanes", type=int, default=0,
                    help="frames in flight per rank, each on its own stream(s) and output buffer "
                         "(tiles.py); 0 at alpha 1 (frames independent): 8 for a band below one "
                         "dispatch round of waves (with 8 hardware queues, see --queues), else 4; "
                         "1 at alpha != 1")
    ap.add_argument("--queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for this process (set before HIP starts); 0: 8 with "
                         "8 lanes for bands below one dispatch round of waves, else the "
                         "environment's value (4 on the GPU box, HIP's default)")
    ap.add_argument("--parts", type=int, default=0,
                    help="interleaved row parts per frame, each on its own HIP stream (tiles.py); "
                         "0: 1 with several lanes, else 2 (one launch's tail overlaps the other's)")
    ap.add_argument("--exact-pass", type=int, default=1, choices=[0, 1, 2],
                    help="pixels the certified walks cannot settle rendered by a second, compacted "
                         "exact pass (vrt_set_exact_pass): 1 automatic (launches of >= 2 rounds of "
                         "resident waves), 2 always, 0 never (in their own lanes)")
    ap.add_argument("--tile-order", type=int, default=1, choices=[0, 1, 2],
                    help="heavy-first tile order of in-lane launches with glass (vrt_set_tile_order): "
                         "1 automatic (launches of at least one dispatch round of waves), 2 every "
                         "launch, 0 off")
    ap.add_argument("--certified", type=int, default=0, choices=[-1, 0, 1],
                    help="certified pixels (vrt_set_certified): 0 automatic, 1 always, -1 never")
    ap.add_argument("--cert-trees", type=int, default=1, choices=[0, 1, 2],
                    help="certified bounce trees of glass pixels (vrt_set_cert_trees): 1 automatic "
                         "(glass-heavy volumes), 2 always, 0 off")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only for the "
                         "multi-rank rehearsal test)")
    ap.add_argument("--rehearse-ranks", type=int, default=1,
                    help="one GPU, one process: time only rank 0's band of a K-way strong split "
                         "(what each GPU of a K-GPU run renders per frame; rays counted over the "
                         "whole frame); a diagnostic of the scaling path, labelled as such")
    ap.add_argument("--rehearse-rank", type=int, default=0,
                    help="with --rehearse-ranks K: time rank R's band instead of rank 0's (block-"
                         "cyclic bands differ by up to one block; the K-GPU frame is the slowest)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per launch of a rank's band (vrt_render_temporal_batch_async, "
                         "alpha 1): 0 automatic, K for a K-way split (each launch then has about a "
                         "whole frame's waves), 8 from K = 7; 1 off")
    ap.add_argument("--rehearse-gather", action="store_true",
                    help="with --rehearse-ranks K --rehearse-rank 0: also do rank 0's local share of the "
                         "per-frame gather (pack its band to RGB8, assemble the K bands into the frame) "
                         "on each frame's lane stream, as the N > 1 run does after its ncclGather")
    ap.add_argument("--compositor", type=int, default=0, choices=[-1, 0, 1],
                    help="with the per-frame gather (or --rehearse-gather): rank 0 renders no band, "
                         "ranks 1..N-1 split every frame and rank 0 receives and assembles it "
                         "(tiles.split_band_spec); 0 automatic (N >= 4 with the gather), 1 on, -1 off")
    ap.add_argument("--row-block", type=int, default=0,
                    help="rows per block of a rank's band (vrt_render_*_blocks_pitched_async, ABI "
                         "v11): rank r renders blocks r, r+N, ... of B adjacent rows; 0: 16 for a "
                         "split frame of one part per lane, else 1 (cyclic rows)")
    ap.add_argument("--same-device", action="store_true",
                    help="test only: every rank on cuda:0 (rehearse N > 1 on a one-GPU box)")
    ap.add_argument("--no-gather", action="store_true",
                    help="N > 1: keep the bands on their ranks in the timed frames (no per-frame "
                         "gather; one gather of the last frame after the timed region); default: "
                         "every frame gathered to rank 0 and assembled there inside the timed region")
    ap.add_argument("--watchdog-s", type=float, default=-1.0,
                    help="dump every thread's Python stack to stderr and exit non-zero after this "
                         "many seconds if the run is still going (0: off; default -1: 300 s when "
                         "WORLD_SIZE > 1, off for one process). SIGUSR1 dumps the stacks at any time")
    ap.add_argument("--pre-idle-ms", type=float, default=0.0,
                    help="diagnostic: idle the synchronised device this long before the timed "
                         "region (clock-ramp experiments)")
    ap.add_argument("--start-events", default="before", choices=["in", "before"],
                    help="where the lanes' GPU-time start events are recorded: just before the wall "
                         "clock starts, on the idle device (before, default: instrumentation stays "
                         "out of the timed region; the 20-frame command 0.0469 -> 0.0455 ms, "
                         "profiles/r05_s48), or inside it (in)")
    ap.add_argument("--frame-events", action="store_true",
                    help="diagnostic: an event after every timed frame on its lane; prints each "
                         "frame's completion time from the first lane start (JSON frame_events_ms)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: the config's frame is split N ways (default); weak (opt-in): N "
                         "ranks render an N-fold taller frame (each a config-sized band)")
    return ap.parse_args()


def host_cores():
    """CPU counts of this host as seen by this process: the affinity mask, lscpu's logical CPUs,
    the cgroup CPU quota (cpu.max) and OMP_NUM_THREADS; the baseline runs on the smallest of the
    ones that are set (on the GPU box the affinity mask lists the whole machine while the job's
    share is its cgroup quota)."""
    import subprocess

    aff = len(os.sched_getaffinity(0))
    try:
        out = subprocess.run(["lscpu", "-p=CPU"], capture_output=True, text=True, timeout=10).stdout
        lscpu = sum(1 for l in out.splitlines() if l and not l.startswith("#"))
    except Exception:
        lscpu = None
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        pass
    omp = int(os.environ["OMP_NUM_THREADS"]) if os.environ.get("OMP_NUM_THREADS", "").isdigit() else None
    use = min(x for x in (aff, quota, omp) if x)
    return dict(threads=use, affinity_cpus=aff, lscpu_cpus=lscpu, cgroup_cpu_quota=quota,
                omp_num_threads=omp)


def cpu_baseline(cam, vox, n, params, budget_s, threads):
    """The oracle (scalar C restatement of voxel.glsl, `port`) on host cores over a bounded sample
    of the same frame: whole frames if they fit the budget, else every k-th row band. It replays
    every DDA step of the reference's walk (the GPU's certified walks skip most of them), so the
    ratio mixes algorithm and hardware. Also returns the last whole oracle frame (float RGBA, or
    None), the checker of the GPU frame in main()."""
    import oracle

    h = cam.height
    t0 = time.perf_counter()
    _, _, c = oracle.render(cam, vox, n, params, row0=0, rows=h // 16, row_step=16, threads=threads)
    probe = time.perf_counter() - t0
    est_frame = probe * 16
    rays = 0
    frames = 0
    frame = None
    t0 = time.perf_counter()
    if est_frame * 1.5 <= budget_s:
        while True:
            frame, _, c = oracle.render(cam, vox, n, params, threads=threads)
            rays += c["primary_rays"] + c["secondary_rays"] + c["shadow_rays"]
            frames += 1
            if time.perf_counter() - t0 + est_frame > budget_s:
                break
        sample = f"{frames} full frame(s)"
    else:
        step = max(2, int(est_frame / budget_s) + 1)
        _, _, c = oracle.render(cam, vox, n, params, row0=0, rows=h // step, row_step=step,
                                threads=threads)
        rays = c["primary_rays"] + c["secondary_rays"] + c["shadow_rays"]
        sample = f"every {step}th row of one frame ({h // step} rows)"
    dt = time.perf_counter() - t0
    return dict(value=rays / dt / 1e6, unit="Mrays/s", cores=threads, kind="port",
                sample=f"oracle/vrt_oracle.c -O3 (exact walks), {threads} threads, {sample}, "
                       f"{dt:.1f} s"), frame


def lib_sha256():
    """SHA-256 of the loaded product library (profiles are stamped with it)."""
    import hashlib

    from voxelraytracer_amd import abi

    with open(abi.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


# resident waves of the certified pass on one MI355X: 256 CUs x 4 SIMDs x 7 waves
# (vrt_context.cpp's wave_slots; a band below one such round is latency-bound)
WAVE_SLOTS = 256 * 4 * 7


def pipeline_shape(args, world: int):
    """(lanes, hardware queues) of this rank's frame pipeline, decided before HIP starts. A band
    below one dispatch round of waves (C3 / C2 at 8 ranks: 4 080 waves) is the latency of its
    slowest waves, and 8 frames in flight on 8 hardware queues hide them (C3 k = 8, slowest rank:
    0.0139 -> 0.0085 ms per frame; C2 k = 8 0.0130 -> 0.0111); larger bands and whole frames are
    faster with 4 on 4 (whole C3 0.0387 vs 0.0420; C3 k = 4 0.0149 vs 0.0154; C4 k = 8 0.0236 vs
    0.0275; profiles/r03_s48-r03_s50)."""
    _, _, w, h, _, _, _ = CONFIGS[args.config]
    frame_h = h * world if args.scaling == "weak" else h
    split = max(world, args.rehearse_ranks if world == 1 else 1)
    if compositor_on(args, world):
        split -= 1   # the renderers' split (rank 0 renders nothing)
    rows = -(-frame_h // split)
    waves = -(-w // 8) * -(-rows // 8)
    independent = args.alpha == 1.0
    batch = frame_batch(args, split)
    small = split > 1 and waves * batch < WAVE_SLOTS
    lanes = args.lanes or ((8 if small else 4) if independent else 1)
    queues = args.queues or (8 if small and lanes == 8 else 4)
    return lanes, queues, batch


def compositor_on(args, world: int) -> bool:
    """Whether rank 0 is a compositor (renders no band; tiles.split_band_spec). Automatic with the
    per-frame gather from 4 ranks: rank 0's share of the exchange (its receive and the assembly of
    every frame) is then worth about one band's render, so rank 0 with a band of its own is the
    slowest rank."""
    if args.compositor == -1:
        return False
    gathered = (world > 1 and not args.no_gather) or (world == 1 and args.rehearse_gather)
    if args.compositor == 1:
        return gathered
    return gathered and world >= 4


def frame_batch(args, split: int) -> int:
    """Frames per launch of a rank's band. A band of a K-way split holds 1/K of the frame's waves:
    below a few dispatch rounds its launches are bound by their longest waves and by the hardware
    queues that overlap them, so K frames per launch (at most 8) give every launch
    about a whole frame's waves again. Only for independent frames (RGBA8 output at alpha 1)."""
    if args.batch:
        return args.batch
    if split <= 1 or args.alpha != 1.0 or args.output != "rgba8" or args.scaling != "strong":
        return 1
    # 7-way bands (the compositor split at N = 8): 8 frames per launch beat 7 (slowest C3 band
    # 0.0068 -> 0.0065 ms, C4 0.0214 -> 0.0210; profiles/r05_s44, r05_s45)
    return 8 if split >= 7 else split


def share_ids(ids, count, dev):
    """RCCL unique ids created on rank 0, broadcast to every rank over the job's process group."""
    import torch
    import torch.distributed as dist

    from voxelraytracer_amd.abi import VRT_COMM_ID_BYTES

    buf = torch.zeros(count * VRT_COMM_ID_BYTES, dtype=torch.uint8, device=dev)
    if ids is not None:
        buf.copy_(torch.frombuffer(bytearray(b"".join(ids)), dtype=torch.uint8))
    dist.broadcast(buf, 0)
    raw = bytes(buf.cpu().numpy())
    return [raw[i * VRT_COMM_ID_BYTES:(i + 1) * VRT_COMM_ID_BYTES] for i in range(count)]


def main():
    args = parse()
    # a hung run (e.g. a collective that never completes) shows every thread's stack: on SIGUSR1
    # (the two-rank test sends it before killing the job) and after --watchdog-s
    faulthandler.enable()
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # multi-rank runs are bounded by default: a hang (a collective that never completes) ends the
    # process with every thread's stack on stderr and a non-zero exit, never a silent wait or an
    # in-place restart
    watchdog_s = args.watchdog_s if args.watchdog_s >= 0 else (300.0 if world > 1 else 0.0)

    def watchdog(phase_s=None):
        """(Re-)arm the hang watchdog for the next phase (each phase gets the full budget; a
        healthy but long run is never cut by the sum of its phases), or cancel it (0)."""
        if watchdog_s <= 0:
            return
        if phase_s == 0:
            faulthandler.cancel_dump_traceback_later()
        else:
            faulthandler.dump_traceback_later(phase_s or watchdog_s, exit=True)

    watchdog()
    lanes, queues, batch = pipeline_shape(args, world)
    if args.queues or queues != 4:   # before HIP initialises (the GPU box exports 4)
        os.environ["GPU_MAX_HW_QUEUES"] = str(queues)
    queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    import numpy as np
    import torch
    import torch.distributed as dist

    import voxelraytracer_amd as vrt
    from voxelraytracer_amd.tiles import FrameTiler, GatherLib, broadcast_volume, row_pitch

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and args.gpus > 1:
        raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run")
    if args.same_device:   # test rehearsal of the multi-rank path on a one-GPU box
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # all host-issued work on a dedicated stream, never the null stream (see GPU_MAX_HW_QUEUES)
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    scene, n, w, h, R, T, desc = CONFIGS[args.config]
    # weak: the framebuffer is H*N rows of the same view (N-fold vertical sample density), so every
    # rank renders an H-row cyclic band of the config's size; strong: the config's frame is split
    frame_h = h * world if args.scaling == "weak" else h
    cam = vrt.make_camera(w, h)   # the config's projection (aspect W/H) at any sample density
    cam.height = frame_h
    params = vrt.default_params(R, T)
    atlas = None
    if args.shading == "textured":
        # the reference's own textures (res/textures/*128.png, decoded into a committed fixture by
        # tests/golden/make_atlas_ref.py), or the synthetic atlas with fractional glass alpha
        atlas = (np.load(os.path.join(ROOT, "tests", "golden", "atlas", "atlas_ref128.npz"),
                         allow_pickle=False)["atlas"] if args.atlas == "ref" else vrt.make_atlas())
        params = vrt.textured_params(params, atlas)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    rgba8 = args.output == "rgba8"

    # Volume: built once on rank 0 (main.cpp:218-288), broadcast over RCCL to every GPU, uploaded
    # device-to-device into each rank's context (padded (N+1)^3 layout built on the GPU).
    vox_host = vrt.build_scene(scene, n) if rank == 0 else np.zeros(n ** 3, np.uint8)
    vox_dev = torch.from_numpy(vox_host).to(dev)
    broadcast_volume(vox_dev)
    ren = vrt.Renderer(local)
    ren.set_exact_pass(args.exact_pass)
    ren.set_certified(args.certified)
    if args.cert_trees != 1 or hasattr(ren._lib, "vrt_set_cert_trees"):   # (an ABI < 15 build: A/B only)
        ren.set_cert_trees(args.cert_trees)
    ren.set_tile_order(args.tile_order)
    ren.upload_volume_device(vox_dev.data_ptr(), n, sptr)
    kparams = params   # the kernel's params: textured frames use the atlas uploaded once
    if atlas is not None:
        ren.upload_atlas(atlas)
        kparams = type(params).from_buffer_copy(params)
        kparams.atlas_rgba = None   # the context's atlas: no per-call compare of its bytes

    # u_Time per frame as the reference sets it (main.cpp:343-345: a frame counter, 1 for the first
    # frame): every launch of the timed path takes its frame's number (tiler.k frames requested so
    # far); the counted and the verifying launches below reuse the last frame's. With zero noise
    # it decides only the sign of a zero direction component (RandomizeDirection, voxel.glsl:132-140).
    # The sun stays where "Make day" puts it: the reference's day/night cycle would move
    # it by ~1e-5 degrees per frame at these frame times.
    def set_frame_time(k):
        kparams.time = float(k)

    def launch(row0, rows, step, out, prev, cnt_ptr=0, row_block=1):
        sp = torch.cuda.current_stream(dev).cuda_stream   # the part's stream (FrameTiler)
        # a part may be a row-strided view into the frame (FrameTiler's single-rank mode)
        pitch = row_pitch(out) if out.dim() == 3 else 0
        if rgba8:
            assert prev.dim() != 3 or row_pitch(prev) == pitch, "one pitch for history and output"
            ren.render_temporal_rows_async(cam, kparams, args.alpha, row0, rows, step,
                                           prev.data_ptr(), out.data_ptr(), 0, 0, cnt_ptr, sp,
                                           pitch=pitch, row_block=row_block)
        else:
            ren.render_rows_async(cam, kparams, row0, rows, step, out.data_ptr(), 0, cnt_ptr, sp,
                                  pitch=pitch, row_block=row_block)

    def render_band(row0, rows, step, out, prev, row_block=1):
        set_frame_time(tiler.k)
        launch(row0, rows, step, out, prev, row_block=row_block)

    def launch_ptrs(row0, rows, step, out_ptr, prev_ptr, pitch, sp, row_block=1):
        # the lean form (FrameTiler's precomputed launches): one ctypes call per part launch
        set_frame_time(tiler.k)
        if rgba8:
            ren.render_temporal_rows_async(cam, kparams, args.alpha, row0, rows, step, prev_ptr,
                                           out_ptr, 0, 0, 0, sp, pitch=pitch, row_block=row_block)
        else:
            ren.render_rows_async(cam, kparams, row0, rows, step, out_ptr, 0, 0, sp, pitch=pitch,
                                  row_block=row_block)

    def launch_batch(row0, rows, step, outs, pitch, sp, row_block=1):
        # frame batches (FrameTiler batch > 1): the band of len(outs) frames in one launch
        k0 = tiler.k - len(outs)   # the batch's frames are k0 + 1 .. tiler.k
        ps = []
        for j in range(len(outs)):
            q = type(kparams).from_buffer_copy(kparams)
            q.time = float(k0 + 1 + j)
            ps.append(q)
        set_frame_time(tiler.k)
        ren.render_temporal_batch_async([cam] * len(outs), ps, row0, rows, step, outs, None, sp,
                                        pitch=pitch, row_block=row_block)

    gather = world > 1 and not args.no_gather
    parts = args.parts or (1 if lanes > 1 or gather else 2)
    parts = parts if frame_h % (max(world, args.rehearse_ranks) * parts) == 0 else 1
    if gather and parts != 1:
        raise SystemExit("gathered bands are one launch per frame (--parts 1)")
    # independent frames: at alpha 1 the kernel does not read the history (tiles.py)
    rehearse = args.rehearse_ranks if world == 1 and args.rehearse_ranks > 1 else 0
    if rehearse and args.scaling != "strong":
        raise SystemExit("--rehearse-ranks rehearses the strong split")
    if not 0 <= args.rehearse_rank < max(rehearse, 1):
        raise SystemExit("--rehearse-rank must be one of the rehearsed split's ranks")
    split = max(world, rehearse) > 1
    # block-cyclic bands (16-row blocks) for a split frame rendered as one part per lane: every
    # 8x8 wave covers 8 adjacent frame rows, as in the whole frame, and a 16x8 workgroup's two
    # neighbours in the band are adjacent too (16 vs 8 rows: C4 k = 8 -3 %, C3 k = 4 -5 %, others
    # equal; profiles/r03_s54)
    row_block = args.row_block or (16 if split and parts == 1 else 1)
    compositor = compositor_on(args, world)
    if compositor and (max(world, rehearse) < 3 or row_block < 2 and not gather):
        raise SystemExit("--compositor needs a gathered split of at least 3 ranks")
    exchange = None
    if args.rehearse_gather:
        if not rehearse or args.rehearse_rank != 0 or not rgba8:
            raise SystemExit("--rehearse-gather rehearses rank 0 of a split with RGBA8 output")
        from voxelraytracer_amd.tiles import GatherRehearsal

        exchange = GatherRehearsal(ren, lanes)
    if gather:   # the per-frame exchange: the library's RCCL path, or torch (gloo rehearsal)
        from voxelraytracer_amd.tiles import GatherLib, GatherTorch

        exchange = (GatherLib(ren, lanes, world, rank, lambda ids, n_: share_ids(ids, n_, dev))
                    if args.backend == "nccl" else GatherTorch())
    tiler = FrameTiler(w, frame_h, render_band, dev, world=rehearse or None,
                       rank=args.rehearse_rank if rehearse else None,
                       dtype=torch.uint8 if rgba8 else torch.float32, parts=parts,
                       gather=gather or args.rehearse_gather, lanes=lanes,
                       independent=rgba8 and args.alpha == 1.0 or not rgba8, launch=launch_ptrs,
                       row_block=row_block, exchange=exchange, batch=batch,
                       launch_batch=launch_batch if batch > 1 else None, compositor=compositor)

    # One counted launch per part (outside the timed region, the exact STATS instance): rays and
    # algorithmic bytes per frame and per launch.
    cnt = torch.zeros(len(vrt.COUNTER_NAMES), dtype=torch.int64, device=dev)
    part_bytes = []
    own = None
    count_specs = tiler.specs
    if rehearse:   # the whole frame's rays: every rank's parts of the rehearsed split, own first
        from voxelraytracer_amd.tiles import part_spec, split_band_spec
        order = [args.rehearse_rank] + [r_ for r_ in range(rehearse) if r_ != args.rehearse_rank]
        count_specs = ([split_band_spec(r_, rehearse, frame_h, row_block, compositor) for r_ in order]
                       if row_block > 1 else
                       [part_spec(r_, rehearse, s_, parts, frame_h) for r_ in order
                        for s_ in range(parts)])
    own_cnt = torch.zeros_like(cnt)
    for i_, (row0, rows, step) in enumerate(count_specs):
        if rows == 0:   # a compositor rank 0: no band
            part_bytes.append(0)
            continue
        pc = torch.zeros_like(cnt)
        scratch = torch.zeros((rows, w, 4), dtype=torch.uint8 if rgba8 else torch.float32, device=dev)
        launch(row0, rows, step, scratch, scratch, pc.data_ptr(), row_block)
        torch.cuda.synchronize(dev)
        pcd = vrt.counters_dict(pc.cpu().tolist())
        cnt += pc
        if i_ < parts:   # this rank's own parts (the rehearsed rank's when rehearsing)
            part_bytes.append(vrt.algorithmic_bytes(pcd, 8 if rgba8 else 16))
            own_cnt += pc
    own = vrt.counters_dict(own_cnt.cpu().tolist())
    if world > 1:
        dist.all_reduce(cnt)
    counters = vrt.counters_dict(cnt.cpu().tolist())
    pixel_bytes = 8 if rgba8 else 16
    rays_per_frame = vrt.total_rays(counters)
    bytes_per_frame = vrt.algorithmic_bytes(counters, pixel_bytes)

    # Device warm-up (untimed): frames until --device-warmup-ms of wall time has passed, so the
    # timed frames run at the clock sustained rendering runs at, not at a fresh process's
    t_w = time.perf_counter()
    warm_frames = 0
    while (time.perf_counter() - t_w) * 1e3 < args.device_warmup_ms:
        for _ in range(16):
            tiler.frame()
        warm_frames += 16
        tiler.finish()
        torch.cuda.synchronize(dev)
    device_warmup = {"ms": round((time.perf_counter() - t_w) * 1e3, 1), "frames": warm_frames,
                     "why": "untimed frames before the W warmup frames: the engine clock ramps "
                            "from ~1.9 to ~2.3 GHz over the first ~150 ms of this load "
                            "(DPM; profiles/r03_s2), so a fresh process's first frames run "
                            "~10 % slower than sustained rendering"}
    watchdog()
    for _ in range(args.warmup):
        tiler.frame()
    tiler.finish()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    watchdog()   # the timed frames: scaled with --steps (a 20-frame run takes milliseconds)
    # Timed region: K frames. The device is idle here (synchronised above), so the lane streams
    # start without waiting on the main stream, and the closing device-wide synchronize waits for
    # every lane (no cross-queue joins inside the timed region: each costs a few us of queue
    # latency at both ends of a 20-frame run; profiles/r03_s33). GPU time per frame: from the
    # earliest lane start event to the latest lane end event. With the per-frame gather, each
    # frame's gather and (rank 0) assembly are on its lane stream: inside both clocks.
    lane_st = tiler.lane_streams() or [stream]

    def timed_frames(steps, events=False):
        """(wall seconds, GPU ms per frame, per-frame completion ms) of `steps` frames between a
        synchronised barrier and a synchronize + barrier (max over ranks is taken by the caller)."""
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        if args.pre_idle_ms > 0:
            time.sleep(args.pre_idle_ms * 1e-3)
        tiler.mark_idle()
        ev0 = [torch.cuda.Event(enable_timing=True) for _ in lane_st]
        ev1 = [torch.cuda.Event(enable_timing=True) for _ in lane_st]
        if args.start_events == "before":   # instrumentation outside the wall clock (device idle)
            for e, st in zip(ev0, lane_st):
                e.record(st)
        t0_ = time.perf_counter()
        if args.start_events == "in":
            for e, st in zip(ev0, lane_st):
                e.record(st)
        fev_ = []
        for i_ in range(steps):
            tiler.frame()
            if events and tiler.pending == 0:
                # one event on every stream of the frame just enqueued (its lane counts the warm-up
                # frames too; no part streams: the current stream); its completion is the last of them.
                # Frame batches: after each batch's launch (its last frame)
                sts = (tiler.part_streams[((tiler.k - 1) // tiler.batch) % tiler.lanes] if tiler.part_streams
                       else [torch.cuda.current_stream(dev)])
                evs = []
                for st_ in sts:
                    e = torch.cuda.Event(enable_timing=True)
                    e.record(st_)
                    evs.append(e)
                fev_.append(evs)
        tiler.flush()   # a partial frame batch is launched inside the timed region
        for e, st in zip(ev1, lane_st):
            e.record(st)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0_
        tiler.finish()   # host bookkeeping: every lane is already complete
        gpu_ms = max(a.elapsed_time(b) for a in ev0 for b in ev1) / steps
        return el, gpu_ms, [round(max(min(a.elapsed_time(e) for a in ev0) for e in evs), 4)
                            for evs in fev_] or None

    elapsed, frame_gpu_ms, frame_events_ms = timed_frames(args.steps, args.frame_events)
    # The same frames without the per-frame gather (labelled "render_only"): what the split alone
    # sustains, beside the timed gathered frames above
    render_only = None
    if tiler.gather:
        tiler.exchange_on = False
        ro_el, ro_gpu, _ = timed_frames(args.steps)
        tiler.exchange_on = True
        t_ro = torch.tensor([ro_el, ro_gpu], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t_ro, op=dist.ReduceOp.MAX)
        ro_el, ro_gpu = t_ro.tolist()
        render_only = {"value": round(rays_per_frame * args.steps / ro_el / 1e6, 3),
                       "ms_per_step": round(ro_el / args.steps * 1e3, 4),
                       "kernel_ms_max_over_ranks": round(ro_gpu, 4),
                       "what": "the same timed frames with the per-frame gather and assembly off "
                               "(bands kept on their ranks); not the headline value"}
    # Launch-timing pass (after the timed region, the same FrameTiler path): the mean duration of
    # one render_kernel launch — what rocprofv3 reports per kernel — from the kernels' own device
    # start / end timestamps (vrt_set_launch_timing: hipExtLaunchKernelGGL events; launches of
    # frames in flight overlap, so a launch lasts longer than frame_gpu_ms / parts). Not in the
    # timed region: the per-launch events cost ~8 % of the frame rate (r02 s17).
    lt_frames = max(20, min(args.steps, 200))
    lt_frames -= lt_frames % batch   # whole batches: every launch holds `batch` frames
    ren.set_launch_timing(lt_frames * parts // batch)
    for _ in range(lt_frames):
        tiler.frame()
    tiler.finish()
    lt_total, lt_n = ren.launch_timing()
    ren.set_launch_timing(0)
    launch_ms = lt_total / max(lt_n, 1)
    watchdog()
    # Exchange timing pass (after the timed region; GatherLib only): per frame, device events on its
    # lane stream around the RGB8 pack + ncclGather (from the render's end, so a rank that arrives
    # early also waits there for the slowest rank's band) and around rank 0's assembly
    exchange_t = None
    if tiler.gather and isinstance(tiler.exchange, GatherLib) and not args.rehearse_gather:
        tiler.exchange.timing = []
        for _ in range(max(16, 2 * lanes * batch)):
            tiler.frame()
        tiler.finish()
        torch.cuda.synchronize(dev)
        evs_x = tiler.exchange.timing
        tiler.exchange.timing = None
        exchange_t = (float(np.median([a_.elapsed_time(b_) for a_, b_, _ in evs_x])),
                      float(np.median([b_.elapsed_time(c_) for _, b_, c_ in evs_x])))
    # a compositor rank 0 launches no render: the roofline fields are renderer rank 1's
    own_bytes = vrt.algorithmic_bytes(own, 8 if rgba8 else 16)
    bytes_per_launch = float(np.mean(part_bytes)) * batch   # a launch renders `batch` frames
    renderer_gpu_ms = frame_gpu_ms
    if compositor and world > 1:
        t_r = torch.tensor([launch_ms, bytes_per_launch, own_bytes, frame_gpu_ms], dtype=torch.float64,
                           device=dev)
        dist.broadcast(t_r, 1)
        launch_ms, bytes_per_launch, own_bytes, renderer_gpu_ms = t_r.tolist()
    t = torch.tensor([elapsed, frame_gpu_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, frame_ms_max = t.tolist()

    # Single-frame latency (after the timed region): one frame alone on the device — its lane's
    # launches (certified pass + deferred exact pass; with the per-frame gather also the gather
    # and rank 0's assembly) between device events on that lane, ranks aligned by a barrier —
    # what the reference's blocking GL_TIME_ELAPSED query around its one draw measures
    # (main.cpp:350-356); median of 15. And the drop-in's synchronous call (vrt_render_frame:
    # in-lane exact path, two parts) on one GPU: its kernel_ms (device timestamps).
    lat = []
    for _ in range(15):
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        st_ = tiler.next_stream()
        lane_ = (tiler.k // tiler.batch) % tiler.lanes
        sts_ = tiler.part_streams[lane_] if tiler.part_streams else [st_]   # every part of the frame
        ea = [torch.cuda.Event(enable_timing=True) for _ in sts_]
        eb = [torch.cuda.Event(enable_timing=True) for _ in sts_]
        for e, s_ in zip(ea, sts_):
            e.record(s_)
        tiler.frame()
        tiler.flush()   # frame batches: the frame alone is a batch of one
        for e, s_ in zip(eb, sts_):
            e.record(s_)
        torch.cuda.synchronize(dev)
        lat.append(max(a.elapsed_time(b) for a in ea for b in eb))
    tiler.finish()
    # Frame batches: a frame is launched only when its batch is full, so the batched pipeline's
    # latency is one whole batch alone (request of its first frame to completion of the launch)
    # plus the wait for the batch to fill (batch - 1 frame intervals at the timed frame rate)
    blat = []
    if batch > 1:
        for _ in range(9):
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            lane_ = (tiler.k // tiler.batch) % tiler.lanes
            sts_ = tiler.part_streams[lane_] if tiler.part_streams else [tiler.next_stream()]
            ea = [torch.cuda.Event(enable_timing=True) for _ in sts_]
            eb = [torch.cuda.Event(enable_timing=True) for _ in sts_]
            for e, s_ in zip(ea, sts_):
                e.record(s_)
            for _ in range(batch):
                tiler.frame()
            tiler.flush()
            for e, s_ in zip(eb, sts_):
                e.record(s_)
            torch.cuda.synchronize(dev)
            blat.append(max(a.elapsed_time(b) for a in ea for b in eb))
        tiler.finish()
    lat_t = torch.tensor([float(np.median(lat)), float(np.median(blat)) if blat else 0.0],
                         dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(lat_t, op=dist.ReduceOp.MAX)
    latency = {"frame_latency_ms": round(float(np.median(lat)), 4),
               "frame_latency_ms_max_over_ranks": round(lat_t[0].item(), 4),
               "what": "one frame alone through the timed path (its lane's launches"
                       + (", gather and rank 0's assembly" if tiler.gather else "")
                       + ", device events), median of 15"
                       + ("; a batch of one: see batch_latency_ms for the batched pipeline" if batch > 1 else ""),
               "frames_in_flight": lanes * batch,
               "frames_in_flight_is": "lanes x frames per launch of the timed pipeline (the headline "
                                      "value's frame rate relies on them; the reference's blocking "
                                      "GL timer query keeps about one)"}
    if blat:
        latency["batch_latency_ms_max_over_ranks"] = round(lat_t[1].item(), 4)
        latency["batch_latency_is"] = (f"one batch of {batch} frames alone through the timed path "
                                       "(request of its first frame to the end of its launch and "
                                       "exchange), median of 9")
    if world == 1 and not rehearse and rgba8:
        sync_ms = []
        for _ in range(9):
            _, st_d = ren.render_frame(cam, kparams, args.alpha)
            sync_ms.append(st_d["kernel_ms"])
        latency["sync_frame_kernel_ms"] = round(float(np.median(sync_ms)), 4)
        latency["sync_frame_is"] = ("vrt_render_frame (the drop-in's synchronous call: two "
                                    "interleaved parts, exact path in lane), device timestamps of "
                                    "its launches, median of 9 (the host copy excluded)")

    # Check of the timed path (after all timing): the next `verify_frames` frames through the same
    # FrameTiler (lanes and parts on their streams, tile order seeded by the frames before
    # them, certified walks), each against the exact STATS instance (exact walks, counters on)
    # rendering the same rows from a copy of the same history: the stored bytes (or float frame)
    # must be equal. Single rank: the frames and their histories are kept for the oracle check.
    # With the per-frame gather, rank 0's assembled frame is also compared with an independent
    # assembly of the ranks' bands (torch.distributed gather + index placement, tiles.collect).
    verify = None
    pairs = []   # (history before, frame after) of each verified frame, host copies

    def last_parts():   # this rank's part buffers of the last frame enqueued
        return [tiler.part_rows(tiler.last(), s_) for s_ in range(parts)]

    if not args.no_verify:
        bad = 0
        total = 0
        vc = torch.zeros_like(cnt)
        gather_bad = None
        for _ in range(max(1, args.verify_frames)):
            tiler.finish()
            prev_parts = [t_.clone() for t_ in last_parts()]   # the next frame's history
            prev_full = tiler.last().clone() if world == 1 else None
            got_frame = tiler.frame()
            tiler.finish()
            torch.cuda.synchronize(dev)
            vtime = kparams.time   # this frame's u_Time: the reference launches below reuse it
            for s_, (row0, rows, step) in enumerate(tiler.specs):
                if rows == 0:   # a compositor rank 0: no band
                    continue
                got = last_parts()[s_].contiguous()
                ref = torch.zeros_like(got)
                prev_c = prev_parts[s_].contiguous()
                launch(row0, rows, step, ref, prev_c, vc.data_ptr(), row_block)   # STATS instance
                torch.cuda.synchronize(dev)
                bad += int((got != ref).sum().item())
                total += got.numel()
            if tiler.gather and world > 1:
                full = tiler.collect()
                torch.cuda.synchronize(dev)
                if rank == 0:
                    gather_bad = (gather_bad or 0) + int((full != got_frame).sum().item())
            if prev_full is not None:
                pairs.append((prev_full.cpu().numpy(), tiler.last().cpu().numpy(), vtime))
        own_ok = bad == 0
        if world > 1:   # every rank's parts (a compositor rank 0 has none of its own)
            bt = torch.tensor([bad, total], dtype=torch.int64, device=dev)
            dist.all_reduce(bt)
            bad, total = (int(x) for x in bt.tolist())
        verify = {"verified": own_ok, "frames": max(1, args.verify_frames),
                  "mismatched_elements": bad, "elements": total,
                  "against": "exact walks (STATS instance, counters on) on a copy of the same "
                             "history, every part of " + ("every rank (elements summed)" if world > 1
                                                          else "this rank")}
        if gather_bad is not None:
            verify["gathered_frame_mismatched_elements"] = gather_bad
        seq_ok = True
        if tiler.gather and world > 1:
            # every rank enqueued lane g's gather for the same frames, in the same order per lane
            # communicator (a mismatch would pair different frames' bands, or hang)
            xl = torch.tensor(tiler.exchange_log(), dtype=torch.int64, device=dev)
            x_lo, x_hi = xl.clone(), xl.clone()
            dist.all_reduce(x_lo, op=dist.ReduceOp.MIN)
            dist.all_reduce(x_hi, op=dist.ReduceOp.MAX)
            seq_ok = bool(torch.equal(x_lo, x_hi))
            verify["gather_sequence_equal_all_ranks"] = seq_ok
            verify["gathers_per_lane"] = xl[0::2].tolist()
        ok = torch.tensor([1 if own_ok and not gather_bad and seq_ok else 0], device=dev)
        if world > 1:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        verify["verified_all_ranks"] = bool(ok.item())

    # Bands that stayed on their ranks (--no-gather): one RCCL gather of the last frame to rank 0
    # (after all timing), the delivery a display of the whole frame would do
    collect = None
    if world > 1 and not tiler.gather:
        tiler.finish()
        torch.cuda.synchronize(dev)
        t_c = time.perf_counter()
        full = tiler.collect()
        torch.cuda.synchronize(dev)
        if rank == 0:
            collect = {"rows": int(full.shape[0]), "bytes": int(full.numel() * full.element_size()),
                       "ms": round((time.perf_counter() - t_c) * 1e3, 3),
                       "what": "one gather of every rank's band of the last frame to rank 0 and its "
                               "re-interleave, after the timed region"}

    # Per-rank record (multi-rank runs): what a sub-linear scaling curve needs to name its cause
    per_rank = None
    if world > 1:
        mine = torch.tensor([frame_gpu_ms, launch_ms, float(np.median(lat)),
                             exchange_t[0] if exchange_t else -1.0, exchange_t[1] if exchange_t else -1.0],
                            dtype=torch.float64, device=dev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = []
        for r_, t_ in enumerate(allr):
            v_ = t_.tolist()
            per_rank.append({"rank": r_, "kernel_ms": round(v_[0], 4), "launch_ms": round(v_[1], 4),
                             "frame_latency_ms": round(v_[2], 4),
                             "gather_ms": round(v_[3], 4) if v_[3] >= 0 else None,
                             "assembly_ms": round(v_[4], 4) if v_[4] >= 0 and r_ == 0 else None})
    watchdog(0)

    band_kind = (f"block-cyclic bands of {row_block}-row blocks" if row_block > 1 else
                 "cyclic row bands")
    if compositor:
        band_kind += (" over ranks 1..N-1 (rank 0 renders nothing: it receives and assembles every "
                      "frame, tiles.split_band_spec)")
    gather_how = (("REHEARSAL of rank 0's local share: " + ("the K-1 renderers' bands" if compositor else
                                                             "its band packed to RGB8 and the K bands")
                   + " assembled into the frame per frame, no collective (one GPU)")
                  if args.rehearse_gather else
                  ("RCCL ncclGather over xGMI, one communicator per lane, library assembly kernel"
                   if isinstance(tiler.exchange, GatherLib) else "torch.distributed gather, "
                   f"{args.backend} backend") if tiler.gather else None)
    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = rays_per_frame * args.steps / elapsed / 1e6
        rehearsal = None
        if rehearse:   # one band of a K-way split: value counts that band's own rays only
            own_rays = vrt.total_rays(own)
            rehearsal = {"ranks": rehearse, "rank": args.rehearse_rank, "band_rays_per_frame": own_rays,
                         "whole_frame_equivalent_value": round(value, 3),
                         "whole_frame_equivalent_is": ("the whole frame's rays per rehearsed band time: "
                                                       "what a K-GPU run reports if every rank is as "
                                                       "fast as this one")}
            value = own_rays * args.steps / elapsed / 1e6
        # Roofline of the dominant kernel (render_kernel). Algorithmic bytes are the reference's:
        # 1 B per DDA step of its walk + 2 B per refraction probe + the pixel bytes;
        # the certified walks read only a few texels per pixel, so this is a reference-normalised
        # rate, not a bandwidth. What binds the kernel is VALU issue and dependency latency
        # (valu_issue below); the measured HBM traffic is hbm_frac. Per launch (what rocprofv3
        # reports per kernel): this rank's bytes of one launch over the mean launch duration. With
        # frames in flight, launches overlap (launches_in_flight on average), so the GPU's rate is
        # the per-launch rate times that: this rank's bytes per frame / GPU time per frame.
        # (a compositor rank 0 alone, in a rehearsal, has no launch: no per-launch rate)
        per_launch = bytes_per_launch / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
        in_flight = launch_ms * parts / (renderer_gpu_ms * batch)
        achieved = own_bytes / (renderer_gpu_ms * 1e-3) / 1e9
        lib_hash = lib_sha256()
        traffic = traffic_frame = hbm_frac = None
        valu = None
        prof_note = None
        pmc = os.path.join(ROOT, "profiles", f"pmc_{args.config}_{args.output}.json")
        if os.path.exists(pmc) and world == 1 and args.shading == "color":
            with open(pmc) as f:
                pj = json.load(f)
            if pj.get("lib_sha256") != lib_hash:
                prof_note = (f"{os.path.relpath(pmc, ROOT)} was measured on another build "
                             f"({str(pj.get('lib_sha256'))[:12]} != {lib_hash[:12]}): not used")
            else:
                # the PMC passes run one launch per frame (--parts 1); a frame of `parts`
                # interleaved launches moves the same bytes, split over its launches
                traffic_frame = int(pj["hbm_bytes_per_launch"]) * int(pj.get("parts", 1))
                traffic = traffic_frame // parts
                hbm_frac = round(traffic_frame / (frame_gpu_ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 4)
                if pj.get("valu_insts_per_launch"):
                    # VALU-issue bound of the same frame: a wave64 VALU op takes 2 cycles on a
                    # SIMD32; 1024 SIMDs at the 2.4 GHz peak engine clock (MI355X_MICROARCH.md)
                    insts = pj["valu_insts_per_launch"] * int(pj.get("parts", 1))
                    floor_ms = insts * 2 / (1024 * 2.4e9) * 1e3
                    valu = {"insts_per_frame": int(insts), "issue_bound_ms": round(floor_ms, 4),
                            "frac": round(floor_ms / frame_gpu_ms, 4),
                            "source": os.path.relpath(pmc, ROOT)}
                prof_note = pj.get("source")
        cpu = None
        oracle_check = None
        frame_o = None
        cores = host_cores() if world == 1 else None
        cam1 = vrt.make_camera(w, h)
        if pairs:   # the oracle renders the first verified frame (its u_Time)
            params.time = pairs[0][2]
        if world == 1 and args.cpu_seconds > 0:
            threads = args.cpu_threads or cores["threads"]
            cpu, frame_o = cpu_baseline(cam1, vox_host, n, params, args.cpu_seconds, threads)
            cpu.update({k: v for k, v in cores.items() if k != "threads"})
        if frame_o is None and args.oracle_check and pairs:
            import oracle

            frame_o, _, _ = oracle.render(cam1, vox_host, n, params,
                                          threads=args.cpu_threads or cores["threads"])
        if frame_o is not None and pairs and rgba8:
            # the oracle's frame through the oracle's RGB8 store + temporal filter against the
            # same history, frame by frame: the timed path's stored bytes must be within 1 LSB
            # (colour within 1e-4 may straddle a rounding boundary of x*255)
            import oracle

            worst, off1, nbytes = 0, 0, 0
            frames_o = {params.time: frame_o}   # one oracle frame per verified frame's u_Time
            for prev_np, got_np, t_ in pairs:
                if t_ not in frames_o:
                    params.time = t_
                    frames_o[t_], _, _ = oracle.render(cam1, vox_host, n, params,
                                                       threads=args.cpu_threads or cores["threads"])
                _, cur_o = oracle.temporal(frames_o[t_], prev_np, args.alpha)
                d = np.abs(got_np.astype(np.int16) - cur_o.astype(np.int16))
                worst, off1, nbytes = max(worst, int(d.max())), off1 + int((d == 1).sum()), nbytes + d.size
            oracle_check = {"frames": len(pairs), "u_time": sorted(frames_o), "max_lsb": worst,
                            "bytes_off_by_one": off1, "bytes": nbytes, "ok": worst <= 1}
        out = {
            "metric": "Mrays/sec + achieved HBM GB/s, 1920x1080 @ 128^3 voxels, 4 bounces",
            "value": round(value, 3),
            "value_is": ("rays of the reference's ray tree per frame (primary + secondary stack "
                         "pops + shadow rays, counted by the exact-walk instance) x frames / wall "
                         "time of the timed frames, all ranks: output-equivalent throughput (every ray "
                         "of the reference's tree is still resolved, but the timed certified kernel "
                         "takes fewer DDA steps for most of them: certified walks jump empty space)"),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "verified": None if verify is None else verify["verified_all_ranks"],
            "config": {
                "workload": f"{args.config}: {desc}",
                "scene": scene,
                "volume_n": n,
                "width": w,
                "height": h,
                "frame": f"{w}x{frame_h}" + (f" ({world}x vertical sample density)"
                                             if frame_h != h else ""),
                "max_reflections": R,
                "max_transparencies": T,
                "shading": (f"textured ({'the reference textures, atlas_ref128.npz' if args.atlas == 'ref' else 'synthetic'} 256x256 atlas, 128 px tiles)"
                            if args.shading == "textured" else "colour-only"),
                "output": ("RGB8 ray-trace store + temporal filter (alpha %g) fused, RGBA8 words"
                           % args.alpha) if rgba8 else "float RGBA",
                "parallelism": ((f"{band_kind} x{world} ({args.scaling} scaling) + every frame "
                                 f"gathered to rank 0 ({gather_how}) and assembled there, inside "
                                 "the timed region"
                                 if tiler.gather else
                                 f"{band_kind} x{world} ({args.scaling} scaling), no collective "
                                 "in the timed region (--no-gather: one gather of the last frame "
                                 "after it)")
                                if world > 1 else
                                (f"REHEARSAL on one GPU: only rank {args.rehearse_rank}'s band "
                                 f"({band_kind}) of a {rehearse}-way strong split is rendered and "
                                 "timed; rays counted over the whole frame"
                                 + (f"; with {gather_how}" if args.rehearse_gather else "")
                                 if rehearse else "single GPU, whole frame"))
                               + (f", {batch} frames per launch (frame batches: each launch renders the "
                                  f"band of {batch} consecutive frames, vrt_render_temporal_batch_async)"
                                  if batch > 1 else "")
                               + (f", {lanes} {'batches' if batch > 1 else 'frames'} in flight (lanes)"
                                  if lanes > 1 else "")
                               + f", {parts} interleaved row part{'s' if parts > 1 else ''} per "
                               f"frame on {lanes * parts} HIP stream{'s' if lanes * parts > 1 else ''}",
                "rays_per_frame": rays_per_frame,
                "algorithmic_bytes_per_frame": bytes_per_frame,
                "hw_queues": queues,
            },
            "roofline": {
                "bound": "valu-issue/latency",
                "achieved": round(per_launch, 2),
                "achieved_is": ("reference-normalised algorithmic bytes (1 B per DDA step of the "
                                "reference walk + 2 B per refraction probe + pixel bytes) of one "
                                "launch / its mean duration (launch_ms; not a bandwidth: the certified "
                                "walks read a few texels per pixel). A launch of a large band is the "
                                "certified pass (render_kernel) and its deferred exact pass "
                                "(exact_pass_kernel) on one stream, which rocprofv3 lists as two "
                                "kernels"),
                "achieved_frame_rate": round(achieved, 2),
                "achieved_frame_rate_is": ("the same bytes per frame / GPU time per frame (kernel_ms) "
                                           "= achieved x launches_in_flight: launches of frames in "
                                           "flight overlap"),
                "launches_in_flight": round(in_flight, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(per_launch / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_is": ("measured HBM bytes per launch: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE of a "
                               "one-launch frame (profile stamped with this library's hash) / parts"),
                "traffic_per_frame": traffic_frame,
                "hbm_frac": hbm_frac,
                "hbm_frac_is": "measured HBM bytes per frame / GPU time per frame / 8 TB/s",
                "bytes_per_launch": int(bytes_per_launch),
                "bytes_per_frame": own_bytes,
                "launch_ms": round(launch_ms, 4),
                "launch_ms_is": ("mean launch duration from the device timestamps of its first "
                                 "kernel's start and last kernel's end (hipExtLaunchKernelGGL "
                                 "events, vrt_set_launch_timing) over a pass of the same frames "
                                 "after the timed region"),
                "launches_per_frame": parts,
                "frames_per_launch": batch,
                "lanes": lanes,
                "kernel_ms": round(frame_gpu_ms, 4),
                "kernel_ms_is": (f"GPU time per frame of this rank ({lanes} frame(s) in flight, "
                                 f"{parts} launch(es) per frame): from the earliest start event to "
                                 "the latest end event of the lane streams around the K timed "
                                 "frames / K (with fill and drain of the pipeline; the start events "
                                 "are recorded on the idle device just before the wall clock starts, "
                                 "so the first launch's enqueue is inside)"
                                 if args.start_events == "before" else
                                 f"GPU time per frame of this rank ({lanes} frame(s) in flight, "
                                 f"{parts} launch(es) per frame): from the earliest start event to "
                                 "the latest end event of the lane streams around the K timed "
                                 "frames / K (with fill and drain of the pipeline)"),
                "kernel_ms_max_over_ranks": round(frame_ms_max, 4),
                "rank": (1 if compositor and world > 1 else rank),
                "rank_is": ("the rank the per-launch fields describe (a compositor rank 0 renders "
                            "nothing: renderer rank 1's launches)"),
                "valu_issue": valu,
                "lib_sha256": lib_hash[:16],
                "profile": prof_note,
            },
            "rehearsal": rehearsal,
            "gather": (None if world == 1 else
                       {"per_frame": tiler.gather, "how": gather_how,
                        "band_rows_padded": getattr(tiler, "rmax", None),
                        "compositor": compositor,
                        "bytes_to_rank0_per_frame": (
                            (tiler.exchange.bytes_per_rank(tiler) if isinstance(tiler.exchange, GatherLib)
                             else tiler.rmax * w * (4 if rgba8 else 16)) * (world - 1)
                            if tiler.gather else None),
                        "wire": (("RGB8, 3 B per pixel" if tiler.exchange.rgb8 else "RGBA8/float as rendered")
                                 if isinstance(tiler.exchange, GatherLib) and tiler.exchange.args else
                                 ("as rendered" if tiler.gather else None)),
                        "render_only": render_only,
                        "per_rank": per_rank,
                        "per_rank_is": ("each rank's kernel_ms (GPU time per timed frame), launch_ms, "
                                        "single-frame latency, and from a pass after the timed region "
                                        "the median per-frame gather_ms (device events on the lane "
                                        "stream from the end of the frame's render across the RGB8 "
                                        "pack and ncclGather: includes waiting for the slowest rank) "
                                        "and rank 0's assembly_ms"),
                        "rank0_ingress_gbs": (
                            round(tiler.exchange.bytes_per_rank(tiler) * (world - 1)
                                  / (per_rank[0]["gather_ms"] * 1e-3) / 1e9, 2)
                            if per_rank and per_rank[0]["gather_ms"] and isinstance(tiler.exchange, GatherLib)
                            else None),
                        "rank0_ingress_is": ("bytes every other rank sends rank 0 per frame / rank 0's "
                                             "median gather_ms (an upper bound of the link time: the "
                                             "wait for late ranks is inside)"),
                        "hardware_scaling_measured": ("this run" if world > 1 and args.backend == "nccl"
                                                      and not args.same_device else None)}),
            "latency": latency,
            "device_warmup": device_warmup,
            "frame_events_ms": frame_events_ms,
            "verify": verify,
            "collect": collect,
            "oracle_check": oracle_check,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    ren.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
