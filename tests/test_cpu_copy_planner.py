"""The box-copy kernel planner on the host (no GPU): sbx_copy_kernel_plan runs the same planning
code launch_box_copy does before a launch -- dimension merging, the choice among the masked /
contiguous / direct / LDS-tile / site-block-transpose / block-transpose kernels and their tile
and grid sizing -- on random layouts, so a planner that loops, throws or sizes a grid of zero
blocks shows up here rather than as a hang on a GPU box (round 4's N=4 bench hang was such a
loop).  The kernels' results are checked by tests/test_gpu_copy*.py against the oracle."""
import ctypes
import itertools

import numpy as np
import pytest

import superbblas_amd as sb

_lib = sb._lib
_lib.sbx_copy_kernel_plan.restype = ctypes.c_int
KINDS = {0: "masked", 1: "contiguous", 2: "direct", 3: "tile", 4: "site-block transpose",
         5: "block transpose"}
TYPES = [(0, 0), (1, 1), (2, 2), (3, 3), (0, 1), (1, 0), (2, 3), (3, 2), (0, 2), (1, 3),
         (4, 4), (5, 5)]


def plan(size, src_stride, dst_stride, t0=3, t1=3, add=0, masked=0):
    nd = len(size)
    arr = ctypes.c_longlong * max(nd, 1)
    kind = ctypes.c_int(-2)
    blocks = ctypes.c_longlong(-1)
    rc = _lib.sbx_copy_kernel_plan(nd, arr(*size), arr(*src_stride), arr(*dst_stride), t0, t1,
                                   add, masked, ctypes.byref(kind), ctypes.byref(blocks))
    if rc != 0:
        raise sb.SuperbblasError(_lib.sbx_last_error().decode())
    return kind.value, blocks.value


def packed(size, order):
    """Element strides of `size` laid out with the dimensions in `order` fastest first."""
    st = [0] * len(size)
    s = 1
    for d in order:
        st[d] = s
        s *= size[d]
    return st


def test_empty_box():
    assert plan([0, 4], [1, 0], [1, 0])[0] == -1
    assert plan([5, 0, 3], [1, 5, 0], [1, 5, 0])[0] == -1


def test_identity_layout_is_contiguous():
    for t0, t1 in [(0, 0), (3, 3), (1, 3)]:
        k, b = plan([8, 8, 8, 8, 12], packed([8, 8, 8, 8, 12], range(5)),
                    packed([8, 8, 8, 8, 12], range(5)), t0, t1)
        assert KINDS[k] == "contiguous" and b > 0


def test_masked_is_masked():
    k, b = plan([16, 16, 12], packed([16, 16, 12], [0, 1, 2]), packed([16, 16, 12], [2, 0, 1]),
                masked=1)
    assert KINDS[k] == "masked" and b > 0


def test_rejects_bad_input():
    with pytest.raises(sb.SuperbblasError):
        plan([4], [-1], [1])
    with pytest.raises(sb.SuperbblasError):
        plan([4], [1], [1], t0=3, t1=0)  # complex -> real is not a copy


def test_lattice_permutations_every_kernel():
    """All 24 site-dimension orders of a 4-d lattice with a spin-color block on either side:
    each plan is one of the kernels, with a positive grid."""
    size = [8, 8, 8, 8, 12]
    seen = set()
    for perm in itertools.permutations(range(4)):
        for blk_first in (False, True):
            order_d = ([4] if blk_first else []) + list(perm) + ([] if blk_first else [4])
            for t0, t1, add in [(3, 3, 0), (2, 2, 1), (1, 3, 0)]:
                k, b = plan(size, packed(size, range(5)), packed(size, order_d), t0, t1, add)
                assert k in KINDS and k != 0 and b > 0, (perm, blk_first, k, b)
                seen.add(k)
    assert len(seen) >= 3, seen


@pytest.mark.timeout(120)
def test_random_layouts_fuzz():
    """Random boxes (1-6 dims, sizes 1-69 and powers of two, degenerate ones included, packed or
    padded layouts in random dimension orders, every type pair and Copy/Add): the planner
    returns a kernel and a positive grid for each, within the test's time limit."""
    rng = np.random.default_rng(20261017)
    counts = {}
    for it in range(20000):
        nd = int(rng.integers(1, 7))
        size = [int(rng.integers(1, 70)) if rng.random() < 0.4 else
                int(rng.choice([1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 64])) for _ in range(nd)]
        if int(np.prod(size)) > 1 << 22:
            continue
        o0 = list(rng.permutation(nd))
        o1 = list(rng.permutation(nd))
        s0 = packed(size, o0)
        s1 = packed(size, o1)
        if rng.random() < 0.3:  # padded source: a larger enclosing tensor
            pad = [sz + int(rng.integers(0, 3)) for sz in size]
            s0 = packed(pad, o0)
        if rng.random() < 0.3:
            pad = [sz + int(rng.integers(0, 3)) for sz in size]
            s1 = packed(pad, o1)
        t0, t1 = TYPES[int(rng.integers(len(TYPES)))]
        add = int(rng.integers(2))
        masked = int(rng.random() < 0.05)
        k, b = plan(size, s0, s1, t0, t1, add, masked)
        assert k in KINDS and b > 0, (size, s0, s1, t0, t1, add, masked, k, b)
        if masked:
            assert k == 0
        counts[KINDS[k]] = counts.get(KINDS[k], 0) + 1
    # the fuzz reaches the transposing kernels, not only the gathers
    assert counts.get("tile", 0) + counts.get("site-block transpose", 0) + \
        counts.get("block transpose", 0) > 100, counts
