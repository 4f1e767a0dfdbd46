"""oracle — TEST INFRASTRUCTURE ONLY.

ctypes loader for oracle/build/liboracle.so, the scalar C restatement of res/shaders/voxel.glsl
(oracle/vrt_oracle.c). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package; the product package voxelraytracer_amd never does.
Parity against the reference itself is UNPINNED (the GLSL cannot run here); the restatement is
pinned by hand-derived known-answer tests and by the independent NumPy restatement in
oracle/numpy_oracle.py (see DESIGN.md "Oracle").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

# Interface structs are shared with the C-ABI header (include/vrt.h); import the ctypes mirror
# without importing the product package's runtime (no libvrt.so load happens here).
import importlib.util as _ilu

_spec = _ilu.spec_from_file_location(
    "_vrt_abi_types", os.path.join(_HERE, "..", "voxelraytracer_amd", "abi.py"))
_abi = _ilu.module_from_spec(_spec)
_spec.loader.exec_module(_abi)

Camera, Params, Hit = _abi.Camera, _abi.Params, _abi.Hit
HIT_DTYPE, COUNTER_NAMES, VRT_CNT_COUNT = _abi.HIT_DTYPE, _abi.COUNTER_NAMES, _abi.VRT_CNT_COUNT

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_hash1.restype = C.c_uint32
        L.oracle_hash1.argtypes = [C.c_uint32]
        L.oracle_hash4.restype = C.c_uint32
        L.oracle_hash4.argtypes = [C.c_uint32] * 4
        L.oracle_float_construct.restype = C.c_float
        L.oracle_float_construct.argtypes = [C.c_uint32]
        L.oracle_randomize_direction.restype = None
        L.oracle_randomize_direction.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_float,
                                                 C.c_void_p]
        L.oracle_render.restype = C.c_int
        L.oracle_render.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                    C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_int]
        L.oracle_march_one.restype = C.c_int
        L.oracle_march_one.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_float,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_refract.restype = None
        L.oracle_refract.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_void_p]
        L.oracle_terrain_noise.restype = C.c_int
        L.oracle_terrain_noise.argtypes = [C.c_int, C.c_uint32, C.c_void_p]
        L.oracle_build_scene.restype = C.c_int
        L.oracle_build_scene.argtypes = [C.c_int, C.c_int, C.c_uint32, C.c_void_p]
        L.oracle_get_color.restype = None
        L.oracle_get_color.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_uint8,
                                       C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_temporal.restype = None
        L.oracle_temporal.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_void_p, C.c_void_p,
                                      C.c_uint64]
        L.oracle_temporal_from_raw.restype = None
        L.oracle_temporal_from_raw.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_void_p,
                                               C.c_uint64]
        L.oracle_trace_pixel.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                         C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_trace_pixel.restype = C.c_int
        _lib = L
    return _lib


def hash1(x: int) -> int:
    return lib().oracle_hash1(x)


def hash4(a, b, c, d) -> int:
    return lib().oracle_hash4(a, b, c, d)


def float_construct(m: int) -> float:
    return lib().oracle_float_construct(m)


def randomize_direction(d, p, randomness, seed):
    d = np.asarray(d, np.float32)
    p = np.asarray(p, np.float32)
    out = np.zeros(3, np.float32)
    lib().oracle_randomize_direction(d.ctypes.data, p.ctypes.data, randomness, seed, out.ctypes.data)
    return out


def refract(i, n, eta):
    i = np.asarray(i, np.float32)
    n = np.asarray(n, np.float32)
    out = np.zeros(3, np.float32)
    lib().oracle_refract(i.ctypes.data, n.ctypes.data, eta, out.ctypes.data)
    return out


def build_scene(scene_id: int, n: int, seed: int = 0) -> np.ndarray:
    out = np.zeros(n * n * n, np.uint8)
    rc = lib().oracle_build_scene(scene_id, n, seed, out.ctypes.data)
    if rc != 0:
        raise ValueError(f"oracle_build_scene rc={rc}")
    return out


def terrain_noise(n: int, seed: int = 0) -> np.ndarray:
    out = np.zeros(n * n, np.float32)
    lib().oracle_terrain_noise(n, seed, out.ctypes.data)
    return out


def march_one(vox: np.ndarray, n: int, pos, dir, max_len: float = 100.0):
    vox = np.ascontiguousarray(vox, np.uint8)
    pos = np.asarray(pos, np.float32)
    dir = np.asarray(dir, np.float32)
    vidx = C.c_int32()
    ln = C.c_float()
    pt = np.zeros(3, np.float32)
    nm = np.zeros(3, np.float32)
    steps = C.c_uint32()
    found = lib().oracle_march_one(vox.ctypes.data, n, pos.ctypes.data, dir.ctypes.data, max_len,
                                   C.byref(vidx), C.byref(ln), pt.ctypes.data, nm.ctypes.data,
                                   C.byref(steps))
    return dict(found=bool(found), vidx=vidx.value, len=ln.value, point=pt, normal=nm,
                steps=steps.value)


def render(cam: Camera, vox: np.ndarray, n: int, params: Params, row0: int = 0, rows=None,
           row_step: int = 1, threads: int = 1):
    """Render rows row0 + i*row_step (i < rows). Returns (rgba[rows,W,4], hits[rows,W], counters)."""
    if rows is None:
        rows = cam.height
    w = cam.width
    rgba = np.zeros((rows, w, 4), np.float32)
    hits = np.zeros((rows, w), HIT_DTYPE)
    cnt = np.zeros(VRT_CNT_COUNT, np.uint64)
    vox = np.ascontiguousarray(vox, np.uint8)
    rc = lib().oracle_render(C.addressof(cam), vox.ctypes.data, n, C.addressof(params), row0, rows,
                             row_step, rgba.ctypes.data, hits.ctypes.data, cnt.ctypes.data, threads)
    if rc != 0:
        raise ValueError(f"oracle_render rc={rc}")
    return rgba, hits, {name: int(cnt[i]) for i, name in enumerate(COUNTER_NAMES)}


def temporal(rgba: np.ndarray, prev_rgba8: np.ndarray, alpha: float):
    """RGB8 store + temporal blend of a float frame (oracle_temporal): returns (raw, cur) RGBA8
    arrays shaped like rgba[..., 4]."""
    rgba = np.ascontiguousarray(rgba, np.float32)
    prev = np.ascontiguousarray(prev_rgba8, np.uint8)
    assert rgba.shape == prev.shape and rgba.shape[-1] == 4
    raw = np.empty(rgba.shape, np.uint8)
    cur = np.empty(rgba.shape, np.uint8)
    lib().oracle_temporal(rgba.ctypes.data, prev.ctypes.data, alpha, raw.ctypes.data,
                          cur.ctypes.data, rgba.size // 4)
    return raw, cur


def temporal_from_raw(raw_rgba8: np.ndarray, prev_rgba8: np.ndarray, alpha: float) -> np.ndarray:
    """Temporal blend of already-quantised new pixels (oracle_temporal_from_raw)."""
    raw = np.ascontiguousarray(raw_rgba8, np.uint8)
    prev = np.ascontiguousarray(prev_rgba8, np.uint8)
    assert raw.shape == prev.shape and raw.shape[-1] == 4
    cur = np.empty(raw.shape, np.uint8)
    lib().oracle_temporal_from_raw(raw.ctypes.data, prev.ctypes.data, alpha, cur.ctypes.data,
                                   raw.size // 4)
    return cur


def get_color(atlas, atlas_size: int, tex_size: int, voxel: int, point, index: int,
              textured: bool = True) -> np.ndarray:
    """GetColor of one hit (oracle_get_color)."""
    a = np.ascontiguousarray(atlas, np.uint8)
    pt = np.asarray(point, np.float32)
    out = np.zeros(4, np.float32)
    lib().oracle_get_color(a.ctypes.data, atlas_size, tex_size, int(textured), voxel,
                           pt.ctypes.data, index, out.ctypes.data)
    return out


def trace_pixel(cam: Camera, vox: np.ndarray, n: int, params: Params, px: int, py: int, cap: int = 256):
    """Debug: the reference's ray tree of one pixel (colour-only) as records of 24 floats (code 1:
    a TraceWithShadow call: [1, found, voxel, index, point xyz, len, pos xyz, dir xyz, len0,
    energy, medium, rdepth, tdepth]; code 10: an in-volume refraction: [10, index, crossing xyz,
    len, new dir xyz, new medium, energy, step]) and the pixel's colour."""
    L = lib()
    vox = np.ascontiguousarray(vox, dtype=np.uint8)
    out = np.zeros((cap, 24), np.float32)
    rgba = np.zeros(4, np.float32)
    k = L.oracle_trace_pixel(C.byref(cam), vox.ctypes.data, n, C.byref(params), px, py, out.ctypes.data,
                             cap, rgba.ctypes.data)
    if k < 0:
        raise RuntimeError(f"oracle_trace_pixel: {k}")
    return out[:k], rgba
