"""ctypes mirror of include/vrt.h (the C-ABI drop-in boundary).

The structs here are byte-for-byte the ones in include/vrt.h; tests/test_abi.py checks sizes and
that every function the header declares is exported by the built library.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VRT_LIB") or os.path.join(_HERE, "_lib", "libvrt.so")

VRT_OK = 0
VRT_ERR_INVALID = -1
VRT_ERR_DEVICE = -2
VRT_ERR_NO_VOLUME = -3
VRT_ERR_OOM = -4
VRT_ERR_UNSUPPORTED = -5

VRT_HIT_FLAG_TIE3 = 1
VRT_HIT_FLAG_STEP_CAP = 2
VRT_HIT_FLAG_STACK_FULL = 4
VRT_MAX_STEPS = 4096
VRT_COMM_ID_BYTES = 128

SCENE_TERRAIN = 0
SCENE_GLASS_CUBE = 1
SCENE_REFRACTION = 2
SCENES = {"terrain": SCENE_TERRAIN, "glass_cube": SCENE_GLASS_CUBE, "refraction": SCENE_REFRACTION}

COUNTER_NAMES = (
    "pixels",
    "primary_rays",
    "secondary_rays",
    "shadow_rays",
    "dda_steps",
    "shadow_steps",
    "refraction_probes",
    "tie3",
    "step_cap",
)
VRT_CNT_COUNT = len(COUNTER_NAMES)


class Camera(C.Structure):
    _fields_ = [("inv_pv", C.c_float * 16), ("width", C.c_int32), ("height", C.c_int32)]


class Volume(C.Structure):
    _fields_ = [("voxels", C.POINTER(C.c_uint8)), ("n", C.c_int32)]


class Params(C.Structure):
    _fields_ = [
        ("sun_dir", C.c_float * 3),
        ("time", C.c_float),
        ("ray_noise", C.c_float),
        ("reflection_noise", C.c_float),
        ("refraction_noise", C.c_float),
        ("max_ray_length", C.c_float),
        ("max_reflections", C.c_int32),
        ("max_transparencies", C.c_int32),
        ("color_only", C.c_int32),
        ("reserved0", C.c_int32),
        ("atlas_rgba", C.POINTER(C.c_uint8)),
        ("atlas_size", C.c_int32),
        ("atlas_texture_size", C.c_int32),
    ]


class Hit(C.Structure):
    _fields_ = [
        ("voxel_index", C.c_int32),
        ("ray_length", C.c_float),
        ("steps", C.c_uint32),
        ("flags", C.c_uint32),
    ]


VRT_STATS_COUNTERS = 1   # vrt_stats.request: count (runs the exact-walk instance)


class Stats(C.Structure):
    _fields_ = [
        ("counters", C.c_uint64 * VRT_CNT_COUNT),
        ("kernel_ms", C.c_float),
        ("request", C.c_uint32),
        ("reserved", C.c_float * 2),
    ]


# numpy dtype of one vrt_hit record
HIT_DTYPE = [("voxel_index", "<i4"), ("ray_length", "<f4"), ("steps", "<u4"), ("flags", "<u4")]

# name -> (restype, argtypes): every function include/vrt.h declares
# entry points added after ABI v12 (an older build loaded by VRT_LIB with VRT_LIB_ABI=<its version>
# may lack exactly these)
ADDED_IN = {"vrt_render_temporal_batch_async": 14, "vrt_set_cert_trees": 15}

SIGNATURES = {
    "vrt_abi_version": (C.c_int, []),
    "vrt_create": (C.c_int, [C.c_uint32, C.POINTER(C.c_void_p)]),
    "vrt_create_devices": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p)]),
    "vrt_device_count": (C.c_int, [C.c_void_p]),
    "vrt_device_ordinal": (C.c_int, [C.c_void_p, C.c_int32]),
    "vrt_band_plan": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_void_p]),
    "vrt_band_copy_plan": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]),
    # ABI v12: block-cyclic whole-frame split, one process per GPU (RCCL gather + assembly)
    "vrt_frame_row_block": (C.c_int, [C.c_int32]),
    "vrt_block_band_plan": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_void_p]),
    "vrt_block_copy_plan": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]),
    "vrt_comm_unique_id": (C.c_int, [C.c_void_p, C.c_int32]),
    "vrt_comm_join": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32]),
    "vrt_gather_band_async": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
    "vrt_assemble_blocks_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                            C.c_int32, C.c_int32, C.c_void_p, C.c_int64, C.c_void_p]),
    "vrt_pack_rgb8_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
    "vrt_assemble_blocks_rgb8_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                                 C.c_int32, C.c_int32, C.c_void_p, C.c_int64, C.c_void_p]),
    "vrt_destroy": (None, [C.c_void_p]),
    "vrt_last_error": (C.c_char_p, [C.c_void_p]),
    "vrt_upload_volume": (C.c_int, [C.c_void_p, C.POINTER(Volume)]),
    "vrt_upload_volume_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    "vrt_volume_device_ptr": (C.c_void_p, [C.c_void_p]),
    "vrt_build_scene_device": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_uint32, C.c_void_p]),
    "vrt_debug_packed_volume": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "vrt_debug_collectives": (C.c_int, [C.c_void_p]),
    "vrt_debug_fast_math": (C.c_int, [C.c_void_p, C.c_void_p]),
    "vrt_volume_octants": (C.c_int, [C.c_void_p]),
    "vrt_set_skip_layout": (C.c_int, [C.c_void_p, C.c_int32]),
    "vrt_set_certified": (C.c_int, [C.c_void_p, C.c_int32]),
    "vrt_certified": (C.c_int, [C.c_void_p]),
    "vrt_set_tile_order": (C.c_int, [C.c_void_p, C.c_int32]),
    "vrt_set_exact_pass": (C.c_int, [C.c_void_p, C.c_int32]),
    "vrt_set_cert_trees": (C.c_int, [C.c_void_p, C.c_int32]),
    "vrt_set_launch_timing": (C.c_int, [C.c_void_p, C.c_int32]),
    "vrt_launch_timing": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "vrt_render": (
        C.c_int,
        [C.c_void_p, C.POINTER(Camera), C.POINTER(Params), C.c_void_p, C.c_void_p, C.POINTER(Stats)],
    ),
    "vrt_render_rows_async": (
        C.c_int,
        [
            C.c_void_p,
            C.POINTER(Camera),
            C.POINTER(Params),
            C.c_int32,
            C.c_int32,
            C.c_int32,
            C.c_void_p,
            C.c_void_p,
            C.c_void_p,
            C.c_void_p,
        ],
    ),
    "vrt_render_rows_pitched_async": (
        C.c_int,
        [C.c_void_p, C.POINTER(Camera), C.POINTER(Params), C.c_int32, C.c_int32, C.c_int32,
         C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    ),
    "vrt_render_temporal_rows_pitched_async": (
        C.c_int,
        [C.c_void_p, C.POINTER(Camera), C.POINTER(Params), C.c_float, C.c_int32, C.c_int32,
         C.c_int32, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
         C.c_void_p],
    ),
    "vrt_render_blocks_pitched_async": (
        C.c_int,
        [C.c_void_p, C.POINTER(Camera), C.POINTER(Params), C.c_int32, C.c_int32, C.c_int32,
         C.c_int32, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    ),
    "vrt_render_temporal_blocks_pitched_async": (
        C.c_int,
        [C.c_void_p, C.POINTER(Camera), C.POINTER(Params), C.c_float, C.c_int32, C.c_int32,
         C.c_int32, C.c_int32, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
         C.c_void_p, C.c_void_p],
    ),
    "vrt_render_temporal_batch_async": (
        C.c_int,
        [C.c_void_p, C.c_int32, C.POINTER(Camera), C.POINTER(Params), C.c_int32, C.c_int32,
         C.c_int32, C.c_int32, C.c_int64, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
         C.c_void_p],
    ),
    "vrt_render_temporal_rows_async": (
        C.c_int,
        [C.c_void_p, C.POINTER(Camera), C.POINTER(Params), C.c_float, C.c_int32, C.c_int32,
         C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    ),
    "vrt_render_frame": (
        C.c_int,
        [C.c_void_p, C.POINTER(Camera), C.POINTER(Params), C.c_float, C.c_void_p, C.POINTER(Stats)],
    ),
    "vrt_render_frame_device": (
        C.c_int,
        [C.c_void_p, C.POINTER(Camera), C.POINTER(Params), C.c_float, C.c_void_p,
         C.POINTER(C.c_void_p), C.POINTER(Stats)],
    ),
    "vrt_frame_stream": (C.c_void_p, [C.c_void_p]),
    "vrt_history_reset": (C.c_int, [C.c_void_p]),
    "vrt_upload_atlas": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32]),
    "vrt_debug_randomize": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_float,
                                      C.c_float, C.c_void_p]),
    "vrt_terrain_noise": (C.c_int, [C.c_int32, C.c_uint32, C.c_void_p]),
    "vrt_build_scene": (C.c_int, [C.c_int32, C.c_int32, C.c_uint32, C.c_void_p]),
    "vrt_camera_make": (
        C.c_int,
        [
            C.POINTER(C.c_float * 3),
            C.POINTER(C.c_float * 3),
            C.c_int32,
            C.c_int32,
            C.c_float,
            C.c_float,
            C.c_float,
            C.POINTER(Camera),
        ],
    ),
    "vrt_sun_dir": (None, [C.c_float, C.c_float, C.POINTER(C.c_float * 3)]),
    "vrt_params_default": (None, [C.POINTER(Params)]),
}

_lib = None


class VrtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"vrt error {code}: {msg}")
        self.code = code


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load the HIP library. Fails loudly: there is no CPU fallback for the product path."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `make` (or __graft_entry__.build()); "
            "the voxel ray tracer has no CPU fallback"
        )
    # One HIP runtime per process: if PyTorch is installed, let it load its libamdhip64.so.7 first
    # so the library binds to the same runtime (same soname) instead of /opt/rocm's copy; torch
    # tensors' device pointers are then valid in vrt_render_rows_async.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    older = int(os.environ.get("VRT_LIB_ABI", "0"))   # A/B against an older ABI's build (VRT_LIB)
    for name, (res, args) in SIGNATURES.items():
        if not hasattr(lib, name) and name.startswith("vrt_debug_"):
            continue   # diagnostic entry points exist only in diagnostic builds (make variant)
        if not hasattr(lib, name) and os.environ.get("VRT_LIB") and older and older < ADDED_IN.get(name, 0):
            continue   # an entry point newer than the declared ABI of the VRT_LIB build
        # every other symbol must be there: A/B variants (VRT_LIB) are built from this tree, and an
        # ABI/build mismatch fails here, at load time, not at the first call
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
