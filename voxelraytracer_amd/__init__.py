"""voxelraytracer_amd — MI355X-native drop-in for the per-pixel ray tracer of
Thraix/VoxelRayTracer (res/shaders/voxel.glsl).

The product is the C-ABI library voxelraytracer_amd/_lib/libvrt.so (include/vrt.h): a gfx950
HIP kernel plus the host harness that mirrors src/main.cpp. This module is a thin Python host
over that ABI with the reference's vocabulary (scene, camera, sun, frame, volume).
There is no CPU fallback: constructing a Renderer without the HIP library or a GPU raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .abi import (  # noqa: F401  (re-exported vocabulary)
    COUNTER_NAMES,
    HIT_DTYPE,
    SCENE_GLASS_CUBE,
    SCENE_REFRACTION,
    SCENE_TERRAIN,
    SCENES,
    Camera,
    Params,
    VrtError,
)

# Camera pose of AppScene (main.cpp:171-172) and projection (main.cpp:161): 90 deg, 0.01..100.
DEFAULT_CAM_POS = (-3.45, 2.17, 3.53)
DEFAULT_CAM_ROT = (-33.0, -48.0, 0.0)
FOV_DEG, NEAR, FAR = 90.0, 0.01, 100.0


def lib():
    return abi.load_library()


def build_scene(scene, n: int, seed: int = 0) -> np.ndarray:
    """N^3 uint8 volume, x fastest (main.cpp:218-288). `scene` is a name or SCENE_* id."""
    sid = SCENES[scene] if isinstance(scene, str) else int(scene)
    out = np.zeros(n * n * n, dtype=np.uint8)
    rc = lib().vrt_build_scene(sid, n, seed, out.ctypes.data)
    if rc != 0:
        raise VrtError(rc, "vrt_build_scene")
    return out


def terrain_noise(n: int, seed: int = 0) -> np.ndarray:
    out = np.zeros(n * n, dtype=np.float32)
    rc = lib().vrt_terrain_noise(n, seed, out.ctypes.data)
    if rc != 0:
        raise VrtError(rc, "vrt_terrain_noise")
    return out


def make_camera(width: int, height: int, pos=DEFAULT_CAM_POS, rot=DEFAULT_CAM_ROT,
                fov=FOV_DEG, near=NEAR, far=FAR) -> Camera:
    cam = Camera()
    p = (C.c_float * 3)(*pos)
    r = (C.c_float * 3)(*rot)
    rc = lib().vrt_camera_make(C.byref(p), C.byref(r), width, height, fov, near, far, C.byref(cam))
    if rc != 0:
        raise VrtError(rc, "vrt_camera_make")
    return cam


def sun_dir(time_of_day: float, day_time: float = 50.0):
    out = (C.c_float * 3)()
    lib().vrt_sun_dir(time_of_day, day_time, C.byref(out))
    return tuple(out)


def default_params(max_reflections: int = 1, max_transparencies: int = 2, **kw) -> Params:
    """Bench defaults: "Make day" sun, u_Time=1, noise 0, 100 max length."""
    p = Params()
    lib().vrt_params_default(C.byref(p))
    p.max_reflections = max_reflections
    p.max_transparencies = max_transparencies
    for k, v in kw.items():
        if k == "sun_dir":
            p.sun_dir = (C.c_float * 3)(*v)
        else:
            setattr(p, k, v)
    return p


def counters_dict(values) -> dict:
    return {name: int(values[i]) for i, name in enumerate(COUNTER_NAMES)}


# ---- textured mode (voxel.glsl without _COLOR_ONLY) ---------------------
# Atlas layout (ABI): RGBA8 texels, atlas_size x atlas_size, row r at GL t = (r + 0.5) / size
# (row 0 = bottom, as glTexImage2D consumes rows). Slot (texX, texY) of a material
# (voxel.glsl:64-67) covers columns [texX*ts, (texX+1)*ts) and rows
# [size - (texY+1)*ts, size - texY*ts), which is where GetTextureCoordinate (:167-172) lands.
ATLAS_SLOTS = {"stone": (0, 0), "dirt": (1, 0), "glass": (0, 1), "grass": (1, 1)}


def atlas_slot_rows(size: int, ts: int, tex_x: int, tex_y: int):
    return slice(size - (tex_y + 1) * ts, size - tex_y * ts), slice(tex_x * ts, (tex_x + 1) * ts)


def make_atlas(atlas_size: int = 256, texture_size: int = 128, seed: int = 0) -> np.ndarray:
    """Deterministic synthetic atlas [size, size, 4] uint8 (the reference's PNG textures are not
    shipped): per-slot base colour x value noise; the glass slot has alpha 40..255 with a band of
    fully opaque texels (so both sides of GetColor(hit).a != 1, voxel.glsl:445, occur)."""
    rng = np.random.default_rng(seed)
    a = np.zeros((atlas_size, atlas_size, 4), np.uint8)
    base = {"stone": (128, 128, 128), "dirt": (120, 80, 40), "glass": (170, 220, 255),
            "grass": (30, 160, 40)}
    for name, (tx, ty) in ATLAS_SLOTS.items():
        rs, cs = atlas_slot_rows(atlas_size, texture_size, tx, ty)
        noise = rng.uniform(0.6, 1.0, (texture_size, texture_size, 1))
        rgb = np.clip(np.array(base[name], np.float64) * noise, 0, 255)
        a[rs, cs, :3] = rgb.astype(np.uint8)
        if name == "glass":
            alpha = rng.integers(40, 256, (texture_size, texture_size))
            alpha[:, : texture_size // 8] = 255
            a[rs, cs, 3] = alpha
        else:
            a[rs, cs, 3] = 255
    return a


def load_atlas(texture_dir: str, suffix: str = "128", atlas_size: int = 256) -> np.ndarray:
    """Atlas from the reference's res/textures/{stone,dirt,glass,grass}<suffix>.png (main.cpp:187-
    193), for demos on a host that has them (needs PIL); tests use make_atlas()."""
    from PIL import Image

    a = np.zeros((atlas_size, atlas_size, 4), np.uint8)
    for name, (tx, ty) in ATLAS_SLOTS.items():
        im = np.asarray(Image.open(f"{texture_dir}/{name}{suffix}.png").convert("RGBA"))
        ts = im.shape[0]
        rs, cs = atlas_slot_rows(atlas_size, ts, tx, ty)
        a[rs, cs] = im[::-1]   # image rows are top-down; atlas rows bottom-up
    return a


def textured_params(p: Params, atlas: np.ndarray, texture_size: int = 128) -> Params:
    """Switch params to textured mode with this atlas (kept alive on the Params object)."""
    atlas = np.ascontiguousarray(atlas, np.uint8)
    p.color_only = 0
    p.atlas_rgba = atlas.ctypes.data_as(C.POINTER(C.c_uint8))
    p.atlas_size = atlas.shape[0]
    p.atlas_texture_size = texture_size
    p._atlas_ref = atlas
    return p


def algorithmic_bytes(c: dict, pixel_bytes: int = 16) -> int:
    """1 B per DDA step (both marches) + 2 B per refraction probe + the per-pixel output bytes:
    16 for the float RGBA frame, 8 for the fused temporal RGB8 path (4 B history
    read + 4 B filtered write)."""
    return (c["dda_steps"] + c["shadow_steps"] + 2 * c["refraction_probes"]
            + pixel_bytes * c["pixels"])


def total_rays(c: dict) -> int:
    return c["primary_rays"] + c["secondary_rays"] + c["shadow_rays"]


def band_plan(height: int, k: int, parts: int = 2):
    """The library's whole-frame row plan (vrt_band_plan): ({(band j, part p): (row0, rows,
    row_step, band_row0)}, rows of the largest band). Band j holds frame rows j, j+k, ..."""
    out = np.zeros(k * parts * 4, np.int32)
    cap = lib().vrt_band_plan(height, k, parts, out.ctypes.data)
    if cap < 0:
        raise VrtError(cap, "vrt_band_plan")
    o = out.reshape(k, parts, 4)
    return {(j, p): tuple(int(v) for v in o[j, p]) for j in range(k) for p in range(parts)}, cap


def band_copy_plan(width: int, height: int, k: int, elem_bytes: int):
    """The library's frame-assembly copies (vrt_band_copy_plan): per band j, (dst_offset,
    dst_pitch, src_pitch, row_bytes, rows) of the 2-D copy of band j's packed rows into the frame."""
    out = np.zeros(k * 5, np.int64)
    r = lib().vrt_band_copy_plan(width, height, k, elem_bytes, out.ctypes.data)
    if r < 0:
        raise VrtError(r, "vrt_band_copy_plan")
    return [tuple(int(v) for v in row) for row in out.reshape(k, 5)]


def frame_row_block(k: int) -> int:
    """Rows per block of the bands the whole-frame entry points split a frame into over k devices
    (vrt_frame_row_block: 1 for one device, 16 for k > 1)."""
    return int(lib().vrt_frame_row_block(k))


def block_band_plan(height: int, k: int, row_block: int):
    """vrt_block_band_plan: ([(row0, rows, row_step)] per device, rows of the largest band) of the
    block-cyclic split of `height` rows over k devices in blocks of row_block rows."""
    out = np.zeros(k * 3, np.int32)
    cap = lib().vrt_block_band_plan(height, k, row_block, out.ctypes.data)
    if cap < 0:
        raise VrtError(cap, "vrt_block_band_plan")
    return [tuple(int(v) for v in row) for row in out.reshape(k, 3)], cap


def block_copy_plan(width: int, height: int, k: int, row_block: int, elem_bytes: int):
    """vrt_block_copy_plan: the 2-D copies (band, dst_offset, dst_pitch, src_offset, src_pitch,
    width_bytes, rows) that assemble a frame from k packed block-cyclic band buffers."""
    out = np.zeros(k * 2 * 7, np.int64)
    n = lib().vrt_block_copy_plan(width, height, k, row_block, elem_bytes, out.ctypes.data)
    if n < 0:
        raise VrtError(n, "vrt_block_copy_plan")
    return [tuple(int(v) for v in row) for row in out.reshape(k * 2, 7) if row[6] > 0]


def comm_unique_id() -> bytes:
    """vrt_comm_unique_id: a new RCCL unique id (rank 0 of a one-process-per-GPU job creates one
    per communicator and the job distributes them)."""
    buf = (C.c_uint8 * abi.VRT_COMM_ID_BYTES)()
    r = lib().vrt_comm_unique_id(buf, abi.VRT_COMM_ID_BYTES)
    if r != abi.VRT_COMM_ID_BYTES:
        raise VrtError(r, "vrt_comm_unique_id")
    return bytes(buf)


class Renderer:
    """One vrt_ctx (replaces the GL context + FrameBuffer of the reference). `device` is a HIP
    device ordinal, or a sequence of ordinals: whole frames are then split into row bands across
    them (vrt_create's device mask; a repeated ordinal rehearses the split on one GPU)."""

    def __init__(self, device=0):
        self._lib = lib()
        h = C.c_void_p()
        if isinstance(device, int):
            rc = self._lib.vrt_create(1 << device, C.byref(h))
        else:
            devs = (C.c_int32 * len(device))(*device)
            rc = self._lib.vrt_create_devices(devs, len(device), C.byref(h))
        if rc != 0:
            raise VrtError(rc, f"vrt_create(device={device}) failed (no GPU?)")
        self._h = h
        self.n = None

    def device_count(self) -> int:
        return self._lib.vrt_device_count(self._h)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.vrt_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self._lib.vrt_last_error(self._h)
            raise VrtError(rc, f"{what}: {msg.decode() if msg else ''}")

    def upload_volume(self, voxels: np.ndarray, n: int):
        v = np.ascontiguousarray(voxels, dtype=np.uint8).reshape(-1)
        if v.size != n * n * n:
            raise ValueError("volume size mismatch")
        vol = abi.Volume(v.ctypes.data_as(C.POINTER(C.c_uint8)), n)
        self._check(self._lib.vrt_upload_volume(self._h, C.byref(vol)), "vrt_upload_volume")
        self.n = n

    def upload_volume_device(self, d_voxels: int, n: int, stream: int = 0):
        """Upload from a device buffer (e.g. a torch uint8 CUDA tensor's data_ptr())."""
        self._check(self._lib.vrt_upload_volume_device(self._h, d_voxels, n, stream or None),
                    "vrt_upload_volume_device")
        self.n = n

    def debug_packed_volume(self) -> np.ndarray:
        """The kernel's device volumes [octant][z][y][x] ((N+1)^3 u16 voxel | G << 8 each; 8
        octant volumes, or 1 for N = 1024), for tests."""
        p = self.n + 1
        k = self._lib.vrt_volume_octants(self._h)
        out = np.empty(k * p ** 3, np.uint16)
        self._check(self._lib.vrt_debug_packed_volume(self._h, out.ctypes.data, out.size),
                    "vrt_debug_packed_volume")
        return out.reshape(k, p, p, p)

    def set_skip_layout(self, octants: int):
        """Skip-distance layout of the next upload: 0 auto, 1 centred single volume, 8 octants."""
        self._check(self._lib.vrt_set_skip_layout(self._h, octants), "vrt_set_skip_layout")

    def set_certified(self, mode: int):
        """Certified walks for stats-free colour-only frames: 1 always, -1 never, 0 automatic."""
        self._check(self._lib.vrt_set_certified(self._h, mode), "vrt_set_certified")

    def certified(self) -> bool:
        """Whether the next stats-free colour-only frame uses certified walks."""
        return self._lib.vrt_certified(self._h) == 1

    def set_tile_order(self, on):
        """Heavy-first tile order for stats-free launches: False/0 off, True/1 automatic (default:
        launches of at least one dispatch round of waves), 2 every launch. Images are identical."""
        self._check(self._lib.vrt_set_tile_order(self._h, int(on)), "vrt_set_tile_order")

    def set_exact_pass(self, mode):
        """Deferred exact pass for certified launches: 0/False off, 1/True automatic (default:
        bands of at least two rounds of resident waves), 2 always. Images are identical."""
        self._check(self._lib.vrt_set_exact_pass(self._h, int(mode)), "vrt_set_exact_pass")

    def set_cert_trees(self, mode):
        """Certified bounce trees of glass pixels (ABI v15): 1 automatic (default: glass-heavy
        volumes), 2 always, 0 off. Images are identical."""
        self._check(self._lib.vrt_set_cert_trees(self._h, int(mode)), "vrt_set_cert_trees")

    def volume_device_ptr(self) -> int:
        return self._lib.vrt_volume_device_ptr(self._h) or 0

    def render(self, cam: Camera, params: Params, want_hits: bool = True, counters: bool = True):
        """Synchronous frame: returns (rgba[H,W,4] float32, hits[H,W] structured or None, stats).
        Hit records or counters run the exact-walk instance; with neither, the fast instance
        renders and stats holds kernel_ms only."""
        w, h = cam.width, cam.height
        rgba = np.empty((h, w, 4), dtype=np.float32)
        hits = np.empty((h, w), dtype=HIT_DTYPE) if want_hits else None
        st = abi.Stats()
        st.request = abi.VRT_STATS_COUNTERS if counters else 0
        self._check(
            self._lib.vrt_render(self._h, C.byref(cam), C.byref(params), rgba.ctypes.data,
                                 hits.ctypes.data if want_hits else None, C.byref(st)),
            "vrt_render",
        )
        stats = counters_dict(st.counters)
        stats["kernel_ms"] = float(st.kernel_ms)
        return rgba, hits, stats

    def render_rows_async(self, cam: Camera, params: Params, row0: int, rows: int, row_step: int,
                          d_out: int, d_hit: int = 0, d_counters: int = 0, stream: int = 0,
                          pitch: int = 0, row_block: int = 1):
        """Band render into device pointers (e.g. torch tensors' data_ptr()) on a HIP stream.
        pitch: pixels from one band row to the next (0 = width: a compact band buffer).
        row_block > 1: block-cyclic band (ABI v11): band row i is frame row
        row0 + (i // row_block) * row_step + i % row_block."""
        if row_block != 1:
            self._check(
                self._lib.vrt_render_blocks_pitched_async(
                    self._h, C.byref(cam), C.byref(params), row0, rows, row_step, row_block,
                    pitch or cam.width, d_out, d_hit or None, d_counters or None, stream or None),
                "vrt_render_blocks_pitched_async",
            )
            return
        if pitch:
            self._check(
                self._lib.vrt_render_rows_pitched_async(
                    self._h, C.byref(cam), C.byref(params), row0, rows, row_step, pitch, d_out,
                    d_hit or None, d_counters or None, stream or None),
                "vrt_render_rows_pitched_async",
            )
            return
        self._check(
            self._lib.vrt_render_rows_async(self._h, C.byref(cam), C.byref(params), row0, rows,
                                            row_step, d_out, d_hit or None, d_counters or None,
                                            stream or None),
            "vrt_render_rows_async",
        )

    def render_temporal_rows_async(self, cam: Camera, params: Params, alpha: float, row0: int,
                                   rows: int, row_step: int, d_prev: int, d_cur: int,
                                   d_raw: int = 0, d_hit: int = 0, d_counters: int = 0,
                                   stream: int = 0, pitch: int = 0, row_block: int = 1):
        """Band render with the fused temporal filter + RGB8 store (vrt_render_temporal_rows_async)
        into device RGBA8 buffers (e.g. torch uint8 [rows, W, 4] tensors' data_ptr()). pitch:
        pixels from one band row to the next in every buffer (0 = width). row_block > 1:
        block-cyclic band (vrt_render_temporal_blocks_pitched_async, ABI v11)."""
        if row_block != 1:
            self._check(
                self._lib.vrt_render_temporal_blocks_pitched_async(
                    self._h, C.byref(cam), C.byref(params), alpha, row0, rows, row_step,
                    row_block, pitch or cam.width, d_prev, d_cur, d_raw or None, d_hit or None,
                    d_counters or None, stream or None),
                "vrt_render_temporal_blocks_pitched_async",
            )
            return
        if pitch:
            self._check(
                self._lib.vrt_render_temporal_rows_pitched_async(
                    self._h, C.byref(cam), C.byref(params), alpha, row0, rows, row_step, pitch,
                    d_prev, d_cur, d_raw or None, d_hit or None, d_counters or None,
                    stream or None),
                "vrt_render_temporal_rows_pitched_async",
            )
            return
        self._check(
            self._lib.vrt_render_temporal_rows_async(
                self._h, C.byref(cam), C.byref(params), alpha, row0, rows, row_step, d_prev, d_cur,
                d_raw or None, d_hit or None, d_counters or None, stream or None),
            "vrt_render_temporal_rows_async",
        )

    def render_temporal_batch_async(self, cams, params, row0: int, rows: int, row_step: int,
                                    d_curs, d_raws=None, stream: int = 0, pitch: int = 0,
                                    row_block: int = 1):
        """The same band of len(cams) frames in one launch at alpha 1 (vrt_render_temporal_batch_async,
        ABI v14): cams / d_curs (/ d_raws) one per frame, params one Params or one per frame (ABI
        v15: frames whose params differ beyond u_Time take launches of their own, in order)."""
        nf = len(cams)
        if isinstance(params, Params):
            params = [params] * nf
        if len(params) != nf or len(d_curs) != nf or (d_raws is not None and len(d_raws) != nf):
            raise ValueError(f"render_temporal_batch_async: {nf} cameras need as many params, outputs "
                             "(and raw outputs, when given)")
        ca = (Camera * nf)(*cams)
        pa = (Params * nf)(*params)
        cur = (C.c_void_p * nf)(*d_curs)
        raw = (C.c_void_p * nf)(*d_raws) if d_raws else None
        self._check(
            self._lib.vrt_render_temporal_batch_async(self._h, nf, ca, pa, row0, rows, row_step, row_block,
                                                      pitch or cams[0].width, cur, raw, stream or None),
            "vrt_render_temporal_batch_async",
        )

    def render_frame(self, cam: Camera, params: Params, alpha: float = 1.0, counters: bool = False):
        """main.cpp's frame loop with the history in the context (vrt_render_frame): returns the
        new filtered frame as rgba8[H,W,4] uint8 and the stats (counters only when asked: they
        run the exact-walk instance)."""
        out = np.empty((cam.height, cam.width, 4), dtype=np.uint8)
        st = abi.Stats()
        st.request = abi.VRT_STATS_COUNTERS if counters else 0
        self._check(self._lib.vrt_render_frame(self._h, C.byref(cam), C.byref(params), alpha,
                                               out.ctypes.data, C.byref(st)), "vrt_render_frame")
        stats = counters_dict(st.counters)
        stats["kernel_ms"] = float(st.kernel_ms)
        return out, stats

    def render_frame_device(self, cam: Camera, params: Params, alpha: float, stream: int = 0,
                            timing: bool = False, counters: bool = False):
        """vrt_render_frame_device: the next filtered frame for display, on the first device,
        ordered on `stream`. Returns (device pointer of the W*H RGBA8 frame, owned by the context
        and valid until the fourth later call; stats dict or None). timing or counters wait for
        the frame (counters run the exact-walk instance); the dict then holds kernel_ms (and the
        counters)."""
        st = abi.Stats() if (timing or counters) else None
        if st is not None:
            st.request = abi.VRT_STATS_COUNTERS if counters else 0
        ptr = C.c_void_p()
        self._check(self._lib.vrt_render_frame_device(self._h, C.byref(cam), C.byref(params), alpha,
                                                      stream or None, C.byref(ptr),
                                                      C.byref(st) if st is not None else None),
                    "vrt_render_frame_device")
        if st is None:
            return ptr.value, None
        stats = counters_dict(st.counters)
        stats["kernel_ms"] = float(st.kernel_ms)
        return ptr.value, stats

    def frame_stream(self) -> int:
        """vrt_frame_stream: the HIP stream that produced the last device frame of a stream = 0
        (NULL) render_frame_device call; consume that frame there."""
        return self._lib.vrt_frame_stream(self._h) or 0

    def set_launch_timing(self, launches: int):
        """vrt_set_launch_timing: device start/end timestamps for the next `launches` async band
        launches (0: off)."""
        self._check(self._lib.vrt_set_launch_timing(self._h, int(launches)), "vrt_set_launch_timing")

    def launch_timing(self):
        """vrt_launch_timing: (sum of the recorded launches' kernel durations in ms, launches)."""
        total, n = C.c_double(), C.c_uint64()
        self._check(self._lib.vrt_launch_timing(self._h, C.byref(total), C.byref(n)),
                    "vrt_launch_timing")
        return total.value, n.value

    def debug_collectives(self):
        """vrt_debug_collectives: this one-device context takes the multi-GPU path through RCCL
        (one-rank communicator: ncclBroadcast of the volume, ncclGather of the band)."""
        self._check(self._lib.vrt_debug_collectives(self._h), "vrt_debug_collectives")

    def history_reset(self):
        """Key F (main.cpp:417-421): the last ray-traced frame becomes the temporal history."""
        self._check(self._lib.vrt_history_reset(self._h), "vrt_history_reset")


    def upload_atlas(self, atlas: np.ndarray):
        """Textured mode's atlas ([S, S, 4] uint8, row 0 = bottom) into the context."""
        a = np.ascontiguousarray(atlas, np.uint8)
        self._check(self._lib.vrt_upload_atlas(self._h, a.ctypes.data, a.shape[0]),
                    "vrt_upload_atlas")


    def debug_randomize(self, dirs: np.ndarray, pos: np.ndarray, randomness: float,
                        seed: float) -> np.ndarray:
        """The kernel's RandomizeDirection on [n, 3] inputs (vrt_debug_randomize), for tests."""
        d = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        p = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
        out = np.empty_like(d)
        self._check(self._lib.vrt_debug_randomize(self._h, d.ctypes.data, p.ctypes.data, len(d),
                                                  randomness, seed, out.ctypes.data),
                    "vrt_debug_randomize")
        return out


    def comm_join(self, ids, nranks: int, rank: int):
        """vrt_comm_join: one RCCL communicator per id (a list of VRT_COMM_ID_BYTES-byte ids), this
        context's device as `rank` of `nranks` (blocks until every rank joined each one)."""
        blob = b"".join(ids)
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        self._check(self._lib.vrt_comm_join(self._h, buf, len(ids), nranks, rank), "vrt_comm_join")

    def gather_band_async(self, comm: int, d_band: int, nbytes: int, d_gathered: int, stream: int):
        """vrt_gather_band_async: ncclGather of nbytes from every rank's d_band to rank 0's
        d_gathered (nranks x nbytes) on communicator `comm`, enqueued on `stream`."""
        self._check(self._lib.vrt_gather_band_async(self._h, comm, d_band, nbytes, d_gathered or None,
                                                    stream or None), "vrt_gather_band_async")

    def assemble_blocks_async(self, d_bands: int, k: int, band_rows_cap: int, width: int, height: int,
                              row_block: int, d_frame: int, frame_pitch: int, stream: int):
        """vrt_assemble_blocks_async: the frame's rows from k gathered block-cyclic bands."""
        self._check(self._lib.vrt_assemble_blocks_async(self._h, d_bands, k, band_rows_cap, width, height,
                                                        row_block, d_frame, frame_pitch, stream or None),
                    "vrt_assemble_blocks_async")

    def pack_rgb8_async(self, d_rgba8: int, pixels: int, d_rgb8: int, stream: int):
        """vrt_pack_rgb8_async: RGBA8 words -> 3-byte pixels (the RGB8 wire format of a gather)."""
        self._check(self._lib.vrt_pack_rgb8_async(self._h, d_rgba8, pixels, d_rgb8, stream or None),
                    "vrt_pack_rgb8_async")

    def assemble_blocks_rgb8_async(self, d_bands: int, k: int, band_rows_cap: int, width: int, height: int,
                                   row_block: int, d_frame: int, frame_pitch: int, stream: int):
        """vrt_assemble_blocks_rgb8_async: the frame's RGBA8 rows from k gathered RGB8 bands."""
        self._check(self._lib.vrt_assemble_blocks_rgb8_async(self._h, d_bands, k, band_rows_cap, width, height,
                                                             row_block, d_frame, frame_pitch, stream or None),
                    "vrt_assemble_blocks_rgb8_async")

    def build_scene_device(self, scene: str, n: int, seed: int = 0, stream: int = 0):
        """Build a scene's volume on the device (vrt_build_scene_device) and make it current."""
        self._check(self._lib.vrt_build_scene_device(self._h, SCENES[scene], n, seed,
                                                     stream or None), "vrt_build_scene_device")
        self.n = n
