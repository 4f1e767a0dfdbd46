"""CPU model of the heavy-first tile order's bookkeeping (vrt_render.hip ordered_tile /
order_record, vrt_context.cpp tile_order_begin), checked over many launches with random heavy
patterns and random completion orders: every tile is rendered exactly once per launch, and every
slot keeps its tile's residue mod 8 (the XCD the tile rendered on before). The GPU side of the
same property is tests/test_gpu_tile_order.py (in-place alpha 0.5 frames, where a tile rendered
twice or never would change the image)."""
import random

import pytest

CLASSES = 8
DIV = 4   # VRT_ORD_DIV


class Band:
    """The order buffer of one band: 3 counter sets x 8 classes, 2 rank sets, 2 list sets."""

    def __init__(self, tiles):
        self.tiles = tiles
        self.q = (tiles + CLASSES * DIV - 1) // (CLASSES * DIV)
        self.ctr = [[0] * CLASSES for _ in range(3)]
        self.rank = [[0] * tiles for _ in range(2)]
        self.lst = [[None] * (tiles + CLASSES) for _ in range(2)]
        self.epoch = 0

    def ordered_tile(self, L, ord_r, ctr_r, ctr_z):
        cap = CLASSES * self.q
        if L < cap:
            r, j = L % CLASSES, L // CLASSES
            if j == 0:
                self.ctr[ctr_z][r] = 0
            n = min(self.ctr[ctr_r][r], self.q)
            return self.lst[ord_r][(n - 1 - j) * CLASSES + r] if j < n else None
        t = L - cap
        rk = self.rank[ord_r][t]
        return None if 1 <= rk <= self.q else t

    def order_file(self, tile, heavy, ord_w, ctr_w):
        rank = 0
        if heavy:
            r = tile % CLASSES
            k = self.ctr[ctr_w][r]
            self.ctr[ctr_w][r] += 1
            self.lst[ord_w][k * CLASSES + r] = tile
            rank = k + 1
        self.rank[ord_w][tile] = rank

    def launch(self, heavy_prob, rng):
        e = self.epoch
        ord_r, ord_w = e & 1, (e & 1) ^ 1
        ctr_r, ctr_w, ctr_z = e % 3, (e + 1) % 3, (e + 2) % 3
        self.epoch += 1
        slots = CLASSES * self.q + self.tiles
        dispatched = []
        for L in rng.sample(range(slots), slots):   # workgroups run in any order
            t = self.ordered_tile(L, ord_r, ctr_r, ctr_z)
            if t is not None:
                assert L % CLASSES == t % CLASSES, "a tile left its XCD"
                dispatched.append(t)
        assert sorted(dispatched) == list(range(self.tiles)), "every tile exactly once"
        rng.shuffle(dispatched)                      # completion order
        for t in dispatched:
            self.order_file(t, rng.random() < heavy_prob, ord_w, ctr_w)
        return dispatched


@pytest.mark.parametrize("tiles", [1, 7, 8, 9, 63, 64, 130, 8160])
def test_every_tile_once_and_on_its_xcd(tiles):
    rng = random.Random(tiles)
    band = Band(tiles)
    for launch in range(12):
        # light frames, frames whose heavy tiles overflow the first pass, all-heavy frames
        band.launch([0.0, 0.05, 0.2, 0.5, 1.0][launch % 5], rng)


def test_heavy_tiles_start_first_last_finished_first():
    rng = random.Random(1)
    band = Band(512)
    band.launch(0.0, rng)
    heavy = set(rng.sample(range(512), 40))
    # launch 2: file a known completion order with `heavy` marked
    e = band.epoch
    ord_w, ctr_w = (e & 1) ^ 1, (e + 1) % 3
    band.epoch += 1
    done = list(range(512))
    rng.shuffle(done)
    for t in done:
        band.order_file(t, t in heavy, ord_w, ctr_w)
    # launch 3 reads what launch 2 filed: the first pass holds exactly the heavy tiles, each class
    # in reverse completion order
    e = band.epoch
    ord_r, ctr_r, ctr_z = e & 1, e % 3, (e + 2) % 3
    cap = CLASSES * band.q
    first = [band.ordered_tile(L, ord_r, ctr_r, ctr_z) for L in range(cap)]
    assert {t for t in first if t is not None} == heavy
    for r in range(CLASSES):
        cls = [t for L, t in enumerate(first) if t is not None and L % CLASSES == r]
        want = [t for t in reversed(done) if t in heavy and t % CLASSES == r]
        assert cls == want
