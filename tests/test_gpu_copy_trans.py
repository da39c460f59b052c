"""The site-block transpose copy kernel (copy_trans_kernel): the boxes whose source is contiguous
over [R, a U chain, V1] and whose destination is contiguous over [R, V1] -- bit-exact against the
oracle, with partial tiles, outer dims, alpha, Add and conversions, and identical to the general
tile kernel (sbx_tune_set("copy.trans", -1))."""
import numpy as np
import pytest

from _common import index_valued, int_valued, oracle_copy

pytestmark = pytest.mark.gpu


def _vol(d):
    n = 1
    for x in d:
        n *= x
    return n


def _copy(gpu, alpha, o0, from0, size0, dim0, v0, o1, from1, dim1, v1, add=False):
    import torch
    import superbblas_amd as sb
    t0 = torch.from_numpy(v0).to(gpu)
    t1 = torch.from_numpy(v1).to(gpu)
    sb.copy(alpha, [([0] * len(o0), list(dim0))], o0, from0, size0, dim0, [t0],
            [([0] * len(o1), list(dim1))], o1, from1, dim1, [t1],
            copyadd=sb.Add if add else sb.Copy)
    torch.cuda.synchronize()
    return t1.cpu().numpy(), sb.tune_get("copy.last_pair")


def test_trans_lattice_slices(gpu):
    """configs[1]'s permute shape (xyztsc -> slice n of tnsxyzc) at 8^4: the transpose kernel
    runs (read-back 4) and every slice is bit-exact."""
    L, n = 8, 5
    dim0 = [L, L, L, L, 4, 3]
    dim1 = [L, n, 4, L, L, L, 3]
    v0 = index_valued(_vol(dim0), np.complex128)
    ref = np.zeros(_vol(dim1), np.complex128)
    out = ref.copy()
    for k in range(n):
        oracle_copy(1.0, "xyztsc", [0] * 6, dim0, dim0, v0, "tnsxyzc", [0, k, 0, 0, 0, 0, 0],
                    dim1, ref)
        out, kind = _copy(gpu, 1.0, "xyztsc", [0] * 6, dim0, dim0, v0, "tnsxyzc",
                          [0, k, 0, 0, 0, 0, 0], dim1, out)
        assert kind & 4
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))


# source wvabc (c fastest): R = c, U = (b, a), V1 = v; destinations that keep c then v fastest
SHAPES = [
    ("wvabc", [3, 37, 4, 5, 3], "awbvc"),   # 25 + 12 items of v per tile (a partial tile)
    ("wvabc", [2, 64, 4, 16, 3], "bawvc"),  # U = 64 items (192 elements per v item), QT = 8
    ("vabc", [100, 2, 3, 1], "bavc"),       # R = 1 after dropping c
    ("wvab", [5, 300, 2, 3], "wbav"),       # no run (R = 1), U = (b, a)
    ("wvabc", [2, 9, 16, 16, 2], "awbvc"),  # U = 256 items
]


@pytest.mark.parametrize("o0,dim0,o1", SHAPES)
def test_trans_shapes_bitexact(gpu, o0, dim0, o1):
    import superbblas_amd as sb
    dim1 = [dim0[o0.index(c)] for c in o1]
    v0 = index_valued(_vol(dim0), np.complex128)
    v1 = int_valued(_vol(dim1), np.complex128, 3)
    ref = v1.copy()
    oracle_copy(1.0, o0, [0] * len(o0), dim0, dim0, v0, o1, [0] * len(o1), dim1, ref)
    out, kind = _copy(gpu, 1.0, o0, [0] * len(o0), dim0, dim0, v0, o1, [0] * len(o1), dim1,
                      v1.copy())
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))
    # the general tile kernel gives the same bytes
    sb.tune_set("copy.trans", -1)
    try:
        out2, kind2 = _copy(gpu, 1.0, o0, [0] * len(o0), dim0, dim0, v0, o1, [0] * len(o1),
                            dim1, v1.copy())
    finally:
        sb.tune_set("copy.trans", 0)
    assert not kind2 & 4
    assert np.array_equal(out2.view(np.uint8), ref.view(np.uint8))
    if dim0[-1] > 1 or o0 == "wvab":
        assert kind & 12, (o0, o1)  # a transpose kernel (U = 256 items: the block transpose)


@pytest.mark.parametrize("add", [False, True])
@pytest.mark.parametrize("t1", [np.complex128, np.complex64])
def test_trans_alpha_add_conversion(gpu, add, t1):
    o0, dim0, o1 = "wvabc", [3, 37, 4, 5, 3], "awbvc"
    dim1 = [dim0[o0.index(c)] for c in o1]
    v0 = int_valued(_vol(dim0), np.complex128, 1)
    v1 = int_valued(_vol(dim1), t1, 2)
    ref = v1.copy()
    alpha = 2.0 - 1.0j
    oracle_copy(alpha, o0, [0] * 5, dim0, dim0, v0, o1, [0] * 5, dim1, ref, add=add)
    out, kind = _copy(gpu, alpha, o0, [0] * 5, dim0, dim0, v0, o1, [0] * 5, dim1, v1.copy(),
                      add=add)
    assert kind & 4
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))


def test_trans_subbox_falls_back(gpu):
    """A sub-box whose source is not one run over [R, U, V1] takes the general kernel."""
    o0, dim0, o1 = "wvabc", [3, 37, 4, 5, 3], "awbvc"
    dim1 = [dim0[o0.index(c)] for c in o1]
    from0, size0 = [0, 2, 0, 1, 0], [3, 30, 4, 4, 3]
    v0 = index_valued(_vol(dim0), np.complex128)
    v1 = np.zeros(_vol(dim1), np.complex128)
    ref = v1.copy()
    oracle_copy(1.0, o0, from0, size0, dim0, v0, o1, [0] * 5, dim1, ref)
    out, kind = _copy(gpu, 1.0, o0, from0, size0, dim0, v0, o1, [0] * 5, dim1, v1.copy())
    assert not kind & 4
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))


@pytest.mark.parametrize("t0,t1", [(np.complex64, np.complex64), (np.complex64, np.complex128),
                                   (np.float64, np.float64), (np.float32, np.float32),
                                   (np.int32, np.int32), (np.float64, np.complex128),
                                   (np.complex128, np.complex64)])
@pytest.mark.parametrize("o0,dim0,o1", [("wvabc", [3, 37, 4, 5, 2], "awbvc"),
                                        ("wvabc", [2, 64, 4, 16, 3], "bawvc"),
                                        ("wvab", [5, 300, 2, 3], "wbav")])
def test_trans_types_and_pairs(gpu, t0, t1, o0, dim0, o1):
    """Every element type through the transpose kernel; 8-byte elements with paired 16-byte
    accesses where the runs are even (read-back bits 1 / 2; reads paired only for 8-byte
    destinations), single accesses otherwise."""
    dim1 = [dim0[o0.index(c)] for c in o1]
    v0 = index_valued(_vol(dim0), t0) if np.dtype(t0).kind in "fc" else \
        np.arange(_vol(dim0)).astype(t0)
    v1 = np.zeros(_vol(dim1), t1)
    ref = v1.copy()
    oracle_copy(1.0, o0, [0] * len(o0), dim0, dim0, v0, o1, [0] * len(o1), dim1, ref)
    out, kind = _copy(gpu, 1.0, o0, [0] * len(o0), dim0, dim0, v0, o1, [0] * len(o1), dim1, v1)
    if np.dtype(t1).itemsize >= 8:  # (4-byte destinations: runs of 24 elements are too short)
        assert kind & 4
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))
    if np.dtype(t0).itemsize == 8 and np.dtype(t1).itemsize == 8 and dim0[-1] % 2 == 0:
        assert kind & 3 == 3  # even runs of 8-byte elements: paired reads and writes


def test_trans_misaligned_pointers(gpu):
    """complex<float> tensors starting 8 bytes past a 16-byte boundary: single accesses."""
    import torch
    import superbblas_amd as sb
    o0, dim0, o1 = "wvabc", [2, 64, 4, 16, 2], "bawvc"
    dim1 = [dim0[o0.index(c)] for c in o1]
    v0 = index_valued(_vol(dim0), np.complex64)
    ref = np.zeros(_vol(dim1), np.complex64)
    oracle_copy(1.0, o0, [0] * 5, dim0, dim0, v0, o1, [0] * 5, dim1, ref)
    s_buf = torch.zeros(_vol(dim0) + 1, dtype=torch.complex64, device=gpu)
    d_buf = torch.zeros(_vol(dim1) + 1, dtype=torch.complex64, device=gpu)
    s_buf[1:] = torch.from_numpy(v0).to(gpu)
    sb.copy(1.0, [([0] * 5, dim0)], o0, [0] * 5, dim0, dim0, [s_buf[1:]], [([0] * 5, dim1)], o1,
            [0] * 5, dim1, [d_buf[1:]])
    torch.cuda.synchronize()
    assert sb.tune_get("copy.last_pair") == 4
    assert np.array_equal(d_buf[1:].cpu().numpy().view(np.uint8), ref.view(np.uint8))


@pytest.mark.parametrize("t0,t1", [(np.complex64, np.complex64), (np.complex128, np.complex128),
                                   (np.complex64, np.complex128), (np.float64, np.float64)])
@pytest.mark.parametrize("n", [12, 5])
@pytest.mark.parametrize("add", [False, True])
def test_btrans_chain_redistribution(gpu, t0, t1, n, add):
    """The block transpose (read-back 8; | 2 for paired stores) on the chain's three-way
    redistribution tnsxyzc -> pxyztscn (n <-> c <-> xyz) at a reduced lattice, with an odd rhs
    count, Add and conversions; identical to the tile kernel (copy.btrans -1)."""
    import superbblas_amd as sb
    L, T = 8, 6
    o0, dim0 = "tnsxyzc", [T, n, 4, L, L, L, 3]
    o1, dim1 = "pxyztscn", [1, L, L, L, T, 4, 3, n]
    v0 = int_valued(_vol(dim0), t0, 1)
    v1 = int_valued(_vol(dim1), t1, 2)
    ref = v1.copy()
    oracle_copy(1.0, o0, [0] * 7, dim0, dim0, v0, o1, [0] * 8, dim1, ref, add=add)
    out, kind = _copy(gpu, 1.0, o0, [0] * 7, dim0, dim0, v0, o1, [0] * 8, dim1, v1.copy(), add=add)
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))
    if np.dtype(t1).itemsize == 8:
        # 8-byte destinations take the block transpose only with paired stores (no Add)
        assert bool(kind & 8) == (not add), kind
        if not add:
            assert kind & 2, kind
    else:
        assert kind & 8, kind
    sb.tune_set("copy.btrans", -1)
    try:
        out2, kind2 = _copy(gpu, 1.0, o0, [0] * 7, dim0, dim0, v0, o1, [0] * 8, dim1, v1.copy(),
                            add=add)
    finally:
        sb.tune_set("copy.btrans", 0)
    assert not kind2 & 8
    assert np.array_equal(out2.view(np.uint8), ref.view(np.uint8))


@pytest.mark.parametrize("t", [np.float32, np.complex64, np.complex128])
@pytest.mark.parametrize("add", [False, True])
def test_trans_many_items_small_chain(gpu, t, add):
    """A short U chain (NU * R = 4) against a long V1 (1584 items): the tile takes at most 256 V1
    items, so its one element of padding per item stays inside the tile (found by the copy fuzz:
    384-item tiles wrote past it into the destination-offset table)."""
    o0, dim0, o1 = "bad", [48, 33, 4], "dba"
    dim1 = [dim0[o0.index(c)] for c in o1]
    v0 = index_valued(_vol(dim0), t) if np.dtype(t).kind == "c" else np.arange(_vol(dim0)).astype(t)
    v1 = int_valued(_vol(dim1), t, 3)
    ref = v1.copy()
    oracle_copy(1.0, o0, [0] * 3, dim0, dim0, v0, o1, [0] * 3, dim1, ref, add=add)
    out, kind = _copy(gpu, 1.0, o0, [0] * 3, dim0, dim0, v0, o1, [0] * 3, dim1, v1.copy(), add=add)
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))


@pytest.mark.parametrize("o0,dim0,o1", [("vpba", [64, 2, 32, 8], "vabp"),
                                        ("vpba", [16, 2, 32, 8], "vabp"),
                                        ("wvpba", [3, 16, 4, 16, 8], "wvabp")])
def test_btrans_split_keeps_source_run(gpu, o0, dim0, o1):
    """the destination chain of the block transpose split a dimension the
    source chain had already taken in the middle of its run (complex<double>, source a,b,p,v
    fastest first, destination p,b,a,v), so the kernel read the source run as contiguous across
    a broken stride.  Bit-exact against the oracle and the tile kernel (copy.btrans -1)."""
    import superbblas_amd as sb
    dim1 = [dim0[o0.index(c)] for c in o1]
    v0 = index_valued(_vol(dim0), np.complex128)
    v1 = int_valued(_vol(dim1), np.complex128, 3)
    ref = v1.copy()
    oracle_copy(1.0, o0, [0] * len(o0), dim0, dim0, v0, o1, [0] * len(o1), dim1, ref)
    out, kind = _copy(gpu, 1.0, o0, [0] * len(o0), dim0, dim0, v0, o1, [0] * len(o1), dim1,
                      v1.copy())
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8)), kind
    sb.tune_set("copy.btrans", -1)
    try:
        out2, _ = _copy(gpu, 1.0, o0, [0] * len(o0), dim0, dim0, v0, o1, [0] * len(o1), dim1,
                        v1.copy())
    finally:
        sb.tune_set("copy.btrans", 0)
    assert np.array_equal(out2.view(np.uint8), ref.view(np.uint8))


@pytest.mark.parametrize("t", [np.complex64, np.float64, np.complex128])
def test_long_runs_strided_box(gpu, t):
    """Runs longer than half a block-transpose tile with one strided outer dim (the chain's halo
    copies: 4608-element runs into a domain with a halo): the block-transpose planner's halving
    loop never ended when no two items fit a tile (cap 0) -- a host hang.  Bit-exact."""
    o, d0, d1 = "ab", [4, 2000], [5, 2001]
    v0 = index_valued(_vol(d0), t) if np.dtype(t).kind == "c" else np.arange(_vol(d0)).astype(t)
    v1 = int_valued(_vol(d1), t, 3)
    ref = v1.copy()
    oracle_copy(1.0, o, [0, 0], d0, d0, v0, o, [1, 1], d1, ref)
    out, _ = _copy(gpu, 1.0, o, [0, 0], d0, d0, v0, o, [1, 1], d1, v1.copy())
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))
