"""The bounce-stack order of the kernel's exact path (vrt_render.hip exact_pixel) against the
reference's DFS (voxel.glsl:425-452), on random ray trees.

The reference pushes a glass hit's reflection ray, then its refraction ray, and pops the top. The
kernel keeps the ray pushed last in registers and only writes a reflection ray lying under a
refraction ray to its scratch stack. This model checks that both visit the same rays in the same
order and set STACK_FULL on the same hits, for any capacity (the ABI fixes cap = R + T + 1, where
no push is ever dropped; smaller caps exercise the drop rule too).
"""
import random
import zlib

import pytest


def tree_children(rng, node):
    """(reflect?, refract?) for the hit of `node`: a pseudo-random, deterministic tree."""
    r = random.Random(zlib.crc32(f"{rng}/{node}".encode()))
    return r.random() < 0.7, r.random() < 0.6


def reference_order(seed, cap, R, T):
    """voxel.glsl:429-450: stack[0] = primary; while sp: pop, trace, push refl, push refr."""
    stack = [("p", 0, 0)]
    order, full = [], 0
    while stack:
        ray = stack.pop()
        order.append(ray[0])
        name, rd, td = ray
        refl, refr = tree_children(seed, name)
        if refl and rd < R:
            if len(stack) < cap:
                stack.append((name + "r", rd + 1, td))
            else:
                full += 1
        if refr and td < T:
            if len(stack) < cap:
                stack.append((name + "t", rd, td + 1))
            else:
                full += 1
    return order, full


def kernel_order(seed, cap, R, T):
    """exact_pixel: the ray being traced is held outside the stack and counts as an entry."""
    stack = []
    ray = ("p", 0, 0)
    order, full = [ray[0]], 0
    while True:
        name, rd, td = ray
        refl, refr = tree_children(seed, name)
        pr = refl and rd < R
        pt = refr and td < T
        sp = len(stack)
        push_r = pr and sp < cap
        push_t = pt and sp + int(push_r) < cap
        full += int(pr and not push_r) + int(pt and not push_t)
        if push_r and push_t:
            stack.append((name + "r", rd + 1, td))
            ray = (name + "t", rd, td + 1)
        elif push_r:
            ray = (name + "r", rd + 1, td)
        elif push_t:
            ray = (name + "t", rd, td + 1)
        else:
            if not stack:
                break
            ray = stack.pop()
        order.append(ray[0])
    return order, full


@pytest.mark.parametrize("R,T", [(0, 0), (1, 2), (4, 2), (4, 4), (8, 8), (4, 12), (12, 4)])
def test_kernel_stack_order_matches_reference(R, T):
    for seed in range(300):
        for cap in (1, 2, 3, R + T + 1):
            assert kernel_order(seed, cap, R, T) == reference_order(seed, cap, R, T), (seed, cap)


def test_abi_capacity_never_drops():
    """cap = R + T + 1 (vrt_context.cpp validation): STACK_FULL cannot be set."""
    for seed in range(300):
        for R, T in [(4, 4), (8, 8), (12, 4)]:
            assert reference_order(seed, R + T + 1, R, T)[1] == 0


def cert_tree_order(seed, R, T):
    """cert_tree (vrt_render.hip): the ray the reference pops next is held in registers, a
    reflection ray pushed under a refraction ray waits in ONE per-lane LDS slot; a tree that needs a
    second waiting ray gives up (None: the pixel takes the exact path)."""
    ray = ("p", 0, 0)
    order, pending = [ray[0]], None
    while True:
        name, rd, td = ray
        refl, refr = tree_children(seed, name)
        pr, pt = refl and rd < R, refr and td < T
        if pr and pt:
            if pending is not None:
                return None
            pending = (name + "r", rd + 1, td)
            ray = (name + "t", rd, td + 1)
        elif pr:
            ray = (name + "r", rd + 1, td)
        elif pt:
            ray = (name + "t", rd, td + 1)
        else:
            if pending is None:
                break
            ray, pending = pending, None
        order.append(ray[0])
    return order


@pytest.mark.parametrize("R,T", [(0, 0), (1, 2), (4, 2), (4, 4), (8, 8), (12, 4)])
def test_cert_tree_order_matches_reference(R, T):
    """Every tree cert_tree keeps (one waiting ray at most) is folded in the reference's DFS order.
    (The BASELINE frames' glass trees never need a second slot: a refraction ray leaves C1's one-voxel
    wall or C3's glass voxel into air or out of the volume, so only the primary hit has two
    children.)"""
    kept = 0
    for seed in range(400):
        got = cert_tree_order(seed, R, T)
        if got is not None:
            kept += 1
            assert got == reference_order(seed, R + T + 1, R, T)[0], seed
    assert kept > 0
