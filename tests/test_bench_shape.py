"""bench.py's pipeline decisions (no GPU): the compositor rule, frames per launch and lanes of a
K-way split, as the driver's N = 1/2/4/8 runs take them."""
import sys

import pytest

import bench


def shape(argv, world):
    old = sys.argv
    sys.argv = ["bench.py"] + argv
    try:
        args = bench.parse()
    finally:
        sys.argv = old
    return bench.compositor_on(args, world), bench.pipeline_shape(args, world)


@pytest.mark.parametrize("world,comp,batch", [(1, False, 1), (2, False, 2), (3, False, 3),
                                              (4, True, 3), (8, True, 8)])
def test_driver_defaults(world, comp, batch):
    c, (lanes, queues, b) = shape([], world)
    assert c is comp and b == batch and lanes == 4 and queues == 4


def test_flags():
    assert shape(["--no-gather"], 8)[0] is False                     # no gather, no compositor
    assert shape(["--compositor", "-1"], 8)[0] is False
    assert shape(["--compositor", "1"], 3)[0] is True
    assert shape(["--rehearse-ranks", "8", "--rehearse-gather"], 1)[0] is False
    c, (_, _, b) = shape(["--rehearse-ranks", "8", "--rehearse-gather", "--compositor", "1"], 1)
    assert c is True and b == 8                                      # the renderers' 7-way batches
    assert shape(["--alpha", "0.5"], 8)[1][2] == 1                   # dependent frames: no batches
    assert shape(["--batch", "3"], 8)[1][2] == 3
