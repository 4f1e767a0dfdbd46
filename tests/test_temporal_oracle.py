"""Temporal filter + RGB8 framebuffer store (temporal.glsl:18,
main.cpp:363-393, FrameBuffer.cpp:8): the C restatement against hand-derived known answers and
the independent NumPy restatement. Parity with real GL is unpinned at the conversion's
implementation-defined points (ties, NaN), which DESIGN.md pins as round-half-even and NaN -> 0."""
import numpy as np
import pytest

import oracle
from oracle import numpy_oracle as npo


def px(*rgb):
    return np.array([[*rgb, 1.0]], np.float32)


@pytest.mark.parametrize("f,b", [
    (0.0, 0), (1.0, 255), (-3.0, 0), (7.0, 255), (float("nan"), 0), (float("inf"), 255),
    (0.5, 128),                 # 127.5 -> tie -> even 128
    (1.5 / 255.0, 2),           # 1.5 -> tie -> even 2
    (2.5 / 255.0, 2),           # 2.5 -> tie -> even 2
    (1.0 / 255.0, 1), (254.0 / 255.0, 254),
])
def test_unorm8_known_answers(built, f, b):
    raw, cur = oracle.temporal(px(f, f, f), np.zeros((1, 4), np.uint8), 1.0)
    assert list(raw[0]) == [b, b, b, 255]
    assert list(cur[0]) == [b, b, b, 255]
    assert npo.unorm8(np.float32(f)) == b


def test_blend_known_answer(built):
    # 0.25*(200/255) + 0.75*(100/255) = 125/255 in exact arithmetic; float32 rounding keeps
    # the product within the same byte
    _, cur = oracle.temporal(px(200 / 255, 0, 1), np.array([[100, 255, 0, 7]], np.uint8), 0.25)
    assert list(cur[0]) == [125, 191, 64, 255]


def test_c_matches_numpy_random(built):
    rng = np.random.default_rng(7)
    n = 200_000
    f = rng.uniform(-0.2, 1.2, (n, 4)).astype(np.float32)
    # near-tie values: (k + 0.5) / 255 and its float neighbours
    k = rng.integers(0, 255, n // 4)
    t = ((k + 0.5) / 255.0).astype(np.float32)
    f[: n // 4, 0] = t
    f[n // 4: n // 2, 1] = np.nextafter(t, np.float32(2))
    f[n // 2: 3 * n // 4, 2] = np.nextafter(t, np.float32(-1))
    prev = rng.integers(0, 256, (n, 4)).astype(np.uint8)
    for alpha in (1.0, 0.0, 0.5, 0.1, 0.937):
        raw_c, cur_c = oracle.temporal(f, prev, alpha)
        raw_n, cur_n = npo.temporal(f, prev, alpha)
        assert np.array_equal(raw_c, raw_n)
        assert np.array_equal(cur_c, cur_n)
        assert np.array_equal(oracle.temporal_from_raw(raw_c, prev, alpha), cur_c)


def test_alpha_identities(built):
    rng = np.random.default_rng(3)
    f = rng.uniform(0, 1, (5000, 4)).astype(np.float32)
    prev = rng.integers(0, 256, (5000, 4)).astype(np.uint8)
    raw, cur = oracle.temporal(f, prev, 1.0)
    assert np.array_equal(cur, raw)              # u_Alpha = 1 (the slider default): no history
    _, cur0 = oracle.temporal(f, prev, 0.0)
    assert np.array_equal(cur0[:, :3], prev[:, :3])   # u_Alpha = 0: history only
    assert (cur0[:, 3] == 255).all()


def test_ema_sequence_converges(built):
    # a constant input frame pulled into black history with alpha 0.5 approaches the input byte
    f = np.full((1, 4), 200 / 255, np.float32)
    hist = np.zeros((1, 4), np.uint8)
    seq = []
    for _ in range(12):
        _, hist = oracle.temporal(f, hist, 0.5)
        seq.append(int(hist[0, 0]))
    assert seq[0] == 100 and seq == sorted(seq) and seq[-1] in (199, 200)


def test_alpha_one_blend_is_identity(built):
    """temporal.glsl:18 at u_Alpha = 1 on RGB8 texels: 1 * b/255 + 0 * old/255 stores b back for
    every byte b and every history byte (the kernel then skips the history read, vrt_render.hip
    store_pixel)."""
    b = np.arange(256, dtype=np.uint8)
    raw = np.zeros((256, 256, 4), np.uint8)
    raw[..., 0] = b[:, None]
    raw[..., 1] = b[None, :]
    raw[..., 2] = b[::-1, None]
    raw[..., 3] = 255
    prev = np.empty_like(raw)
    prev[..., 0] = b[None, :]
    prev[..., 1] = b[:, None]
    prev[..., 2] = b[None, ::-1]
    prev[..., 3] = 255
    assert np.array_equal(oracle.temporal_from_raw(raw, prev, 1.0), raw)
