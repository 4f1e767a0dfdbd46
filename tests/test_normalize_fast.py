"""CPU: the closed form of RN(1 / RN(sqrt(s))) for s near 1 that the kernel's normalize3 uses
(vrt_render.hip near_one_rsqrt) equals IEEE sqrt + division for every float32 within 1024 ulps of 1
(the kernel's window), restated here bit for bit; and the window is safe by a margin (the closed
form first fails at 2898 ulps above 1)."""
import numpy as np

ONE = 0x3F800000


def closed_form(b: int) -> int:
    if b >= ONE:
        return ONE if b - ONE < 2 else ONE - ((b - ONE) & ~1)
    return ONE + (((((ONE - b) + 1) >> 1) + 1) >> 1)


def ieee(b: int) -> int:
    s = np.array([b], np.uint32).view(np.float32)
    return int((np.float32(1.0) / np.sqrt(s, dtype=np.float32)).view(np.uint32)[0])


def test_window_exhaustive():
    for b in range(ONE - 1024, ONE + 1025):
        assert closed_form(b) == ieee(b), hex(b)


def test_margin():
    assert all(closed_form(b) == ieee(b) for b in range(ONE - 4096, ONE + 2898))
    assert closed_form(ONE + 2898) != ieee(ONE + 2898)
