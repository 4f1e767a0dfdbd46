"""GPU: the kernels' fast correctly rounded reciprocal (vrt_render.hip rcp_newton: the hardware
reciprocal plus one Newton step on its fma residual, 3 VALU instead of the IEEE division's 11) and
square root (sqrt_fix: the hardware square root moved by its fma residuals, without the IEEE
sequence's denormal scaling) equal the IEEE division 1.0f / d and sqrt(s) bit for bit on every
float the kernels use them for, checked over all 2^32 bit patterns (vrt_debug_fast_math); the rest
take the IEEE operations."""
import ctypes as C

import pytest

import voxelraytracer_amd as vrt
from voxelraytracer_amd import abi

pytestmark = pytest.mark.gpu


def test_fast_reciprocal_exhaustive(built):
    with vrt.Renderer(0) as r:
        out = (C.c_uint64 * 7)()
        r._check(r._lib.vrt_debug_fast_math(r._h, out), "vrt_debug_fast_math")
    tested, bad, bad_ones, bad_other, first, sq_tested, sq_bad = list(out)
    print(f"rcp_newton: {tested} patterns taken, {bad} mismatches; all-ones significands "
          f"{bad_ones}, other patterns {bad_other} (division); sqrt_fix: {sq_tested} patterns, "
          f"{sq_bad} mismatches")
    assert tested > 4_000_000_000
    assert bad == 0, f"first mismatch 0x{first:08x}"
    assert sq_tested > 1_300_000_000
    assert sq_bad == 0
