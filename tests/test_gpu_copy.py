"""copy()/permute on the GPU vs the oracle: bit-exact for data movement (north_star)."""
import itertools

import numpy as np
import pytest

from _common import index_valued, int_valued, oracle_copy

pytestmark = pytest.mark.gpu


def _vol(d):
    n = 1
    for x in d:
        n *= x
    return n


def _gpu_local_copy(gpu, alpha, o0, from0, size0, dim0, v0, o1, from1, dim1, v1, co=0, add=False):
    import torch
    import superbblas_amd as sb
    t0 = torch.from_numpy(v0).to(gpu)
    t1 = torch.from_numpy(v1).to(gpu)
    sb.copy(alpha, [([0] * len(o0), list(dim0))], o0, from0, size0, dim0, [t0],
            [([0] * len(o1), list(dim1))], o1, from1, dim1, [t1], co=co,
            copyadd=sb.Add if add else sb.Copy)
    torch.cuda.synchronize()
    return t1.cpu().numpy()


def test_lattice_permute_slices(gpu):
    """The dist.cpp permute benchmark (dist.cpp:237-266): xyztsc -> slice n of tnsxyzc."""
    L, n = 4, 3
    dim0 = [L, L, L, L, 4, 3]
    dim1 = [L, n, 4, L, L, L, 3]
    v0 = index_valued(_vol(dim0), np.complex128)
    v1 = np.zeros(_vol(dim1), np.complex128)
    ref = v1.copy()
    out = v1.copy()
    for k in range(n):
        oracle_copy(1.0, "xyztsc", [0] * 6, dim0, dim0, v0, "tnsxyzc", [0, k, 0, 0, 0, 0, 0],
                    dim1, ref)
        out = _gpu_local_copy(gpu, 1.0, "xyztsc", [0] * 6, dim0, dim0, v0, "tnsxyzc",
                              [0, k, 0, 0, 0, 0, 0], dim1, out)
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))


@pytest.mark.parametrize("dtype", [np.complex128, np.float64, np.complex64, np.float32, np.int32,
                                   np.uint64])
def test_permutations_bitexact(gpu, dtype):
    rng = np.random.default_rng(7)
    labels = "abcde"
    dim = [3, 4, 5, 2, 6]
    for trial in range(12):
        perm = rng.permutation(5)
        o1 = "".join(labels[p] for p in perm)
        dim1 = [dim[p] for p in perm]
        from0 = [int(rng.integers(0, d)) for d in dim]
        size0 = [int(rng.integers(1, d + 1)) for d in dim]
        from1 = [int(rng.integers(0, d)) for d in dim1]
        v0 = index_valued(_vol(dim), dtype)
        v1 = int_valued(_vol(dim1), dtype, seed=trial) if np.dtype(dtype).kind in "fc" else \
            np.arange(_vol(dim1)).astype(dtype)
        ref = v1.copy()
        oracle_copy(1.0, labels, from0, size0, dim, v0, o1, from1, dim1, ref)
        out = _gpu_local_copy(gpu, 1.0, labels, from0, size0, dim, v0, o1, from1, dim1, v1.copy())
        assert np.array_equal(out.view(np.uint8), ref.view(np.uint8)), (trial, o1, from0, size0)


@pytest.mark.parametrize("add", [False, True])
def test_alpha_add_and_conversion(gpu, add):
    labels, dim = "xyzw", [5, 3, 4, 7]
    o1, dim1 = "wzxy", [7, 4, 5, 3]
    for t0, t1 in [(np.complex128, np.complex128), (np.complex64, np.complex128),
                   (np.complex128, np.complex64), (np.float32, np.float64)]:
        v0 = int_valued(_vol(dim), t0, 1)
        v1 = int_valued(_vol(dim1), t1, 2)
        ref = v1.copy()
        alpha = 2.0 - 1.0j if np.dtype(t0).kind == "c" else 2.0
        oracle_copy(alpha, labels, [1, 0, 2, 3], [4, 3, 2, 7], dim, v0, o1, [0, 1, 4, 2], dim1,
                    ref, add=add)
        out = _gpu_local_copy(gpu, alpha, labels, [1, 0, 2, 3], [4, 3, 2, 7], dim, v0, o1,
                              [0, 1, 4, 2], dim1, v1.copy(), add=add)
        assert np.array_equal(out, ref)


def test_fast_to_slow_and_missing_labels(gpu):
    # origin label of size 1 absent in the destination; destination label absent in the origin
    v0 = index_valued(2 * 1 * 5 * 3, np.complex128)
    v1 = int_valued(5 * 4 * 2 * 3, np.complex128)
    for co in (0, 1):
        ref = v1.copy()
        oracle_copy(1.0, "abcd", [0, 0, 1, 0], [2, 1, 3, 3], [2, 1, 5, 3], v0, "cqad",
                    [2, 3, 0, 0], [5, 4, 2, 3], ref, co=co)
        out = _gpu_local_copy(gpu, 1.0, "abcd", [0, 0, 1, 0], [2, 1, 3, 3], [2, 1, 5, 3], v0,
                              "cqad", [2, 3, 0, 0], [5, 4, 2, 3], v1.copy(), co=co)
        assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))


def test_multicomponent_redistribution(gpu):
    """Copy between two different partitions of the same tensor, several components per
    process (the reference's --components mode, contract.cpp:452-461)."""
    import torch
    import superbblas_amd as sb
    dim = [6, 4, 5, 3]
    o = "xyzc"
    v = index_valued(_vol(dim), np.complex128)
    p0 = sb.basic_partitioning(o, dim, [3, 1, 1, 1], "x", 3, 1)
    p1 = sb.basic_partitioning("czyx", [3, 5, 4, 6], [1, 2, 2, 1], "zy", 4, 1)
    # components of the origin: slices of v
    comps0 = []
    for frm, size in p0:
        full = v.reshape(dim)
        sl = full[frm[0]:frm[0] + size[0], frm[1]:frm[1] + size[1], frm[2]:frm[2] + size[2],
                  frm[3]:frm[3] + size[3]]
        comps0.append(torch.from_numpy(np.ascontiguousarray(sl).ravel()).to(gpu))
    comps1 = [torch.zeros(_vol(size), dtype=torch.complex128, device=gpu) for _, size in p1]
    sb.copy(1.0, p0, o, [0] * 4, dim, dim, comps0, p1, "czyx", [0] * 4, [3, 5, 4, 6], comps1)
    torch.cuda.synchronize()
    full1 = v.reshape(dim).transpose(3, 2, 1, 0)
    for (frm, size), c in zip(p1, comps1):
        exp = full1[frm[0]:frm[0] + size[0], frm[1]:frm[1] + size[1], frm[2]:frm[2] + size[2],
                    frm[3]:frm[3] + size[3]]
        assert np.array_equal(c.cpu().numpy(), np.ascontiguousarray(exp).ravel())


def test_periodic_shift(gpu):
    """The z-shift of dist.cpp:268-296: from1[z] = 1 wraps around the periodic lattice."""
    dim = [2, 3, 4, 4, 5, 3]
    o = "tnsxzc"
    v0 = index_valued(_vol(dim), np.complex128)
    v1 = np.zeros_like(v0)
    ref = v1.copy()
    oracle_copy(1.0, o, [0] * 6, dim, dim, v0, o, [0, 0, 0, 0, 1, 0], dim, ref)
    out = _gpu_local_copy(gpu, 1.0, o, [0] * 6, dim, dim, v0, o, [0, 0, 0, 0, 1, 0], dim, v1)
    assert np.array_equal(out, ref)


def test_host_components(gpu):
    """A CPU-context origin (the tests gather to/scatter from host tensors)."""
    import torch
    import superbblas_amd as sb
    dim = [4, 6]
    v0 = index_valued(24, np.complex128)
    t0 = torch.from_numpy(v0)  # host
    t1 = torch.zeros(24, dtype=torch.complex128, device=gpu)
    sb.copy(1.0, [([0, 0], dim)], "ab", [0, 0], dim, dim, [t0], [([0, 0], [6, 4])], "ba", [0, 0],
            [6, 4], [t1])
    torch.cuda.synchronize()
    assert np.array_equal(t1.cpu().numpy(), v0.reshape(4, 6).T.ravel())
    back = torch.zeros(24, dtype=torch.complex128)
    sb.copy(1.0, [([0, 0], [6, 4])], "ba", [0, 0], [6, 4], [6, 4], [t1], [([0, 0], dim)], "ab",
            [0, 0], dim, [back])
    assert np.array_equal(back.numpy(), v0)


def test_copy_masked_zeroing_and_errors(gpu):
    """Copy with masks where the origin does not cover the region: the uncovered destination
    elements are zeroed only where mask1 is nonzero (dist.h:2356-2382 zeroes through a masked
    local_copy); masked-out elements keep their value.  Complex -> real is rejected."""
    import torch
    import superbblas_amd as sb
    n = 8
    dim = [n, 6]
    # origin: two components, the second empty -> rows 4..7 have no origin
    p0 = [([0, 0], [4, 6]), ([4, 0], [0, 6])]
    p1 = [([0, 0], dim)]
    g0 = np.arange(n * 6, dtype=np.float64).reshape(n, 6) + 1
    v0 = [torch.from_numpy(g0[:4].copy().ravel()).to(gpu), torch.zeros(0, dtype=torch.float64, device=gpu)]
    m = ((np.arange(n)[:, None] + np.arange(6)[None, :]) % 3 != 0).astype(np.float32)
    y0 = -np.ones((n, 6))
    v1 = [torch.from_numpy(y0.ravel().copy()).to(gpu)]
    m0 = [torch.from_numpy(m[:4].ravel().copy()).to(gpu), torch.zeros(0, dtype=torch.float32, device=gpu)]
    m1 = [torch.from_numpy(m.ravel().copy()).to(gpu)]
    sb.copy(1.0, p0, "ab", [0, 0], dim, dim, v0, p1, "ab", [0, 0], dim, v1, mask0=m0, mask1=m1)
    torch.cuda.synchronize()
    out = v1[0].cpu().numpy().reshape(n, 6)
    ref = y0.copy()
    ref[:4][m[:4] != 0] = g0[:4][m[:4] != 0]
    ref[4:][m[4:] != 0] = 0
    assert np.array_equal(out, ref)
    # complex -> real is not a supported conversion (blas.h:57-65)
    vc = [torch.zeros(n * 6, dtype=torch.complex128, device=gpu)]
    with pytest.raises(sb.SuperbblasError, match="conversion"):
        sb.copy(1.0, p1, "ab", [0, 0], dim, dim, vc, p1, "ab", [0, 0], dim, v1)
    with pytest.raises(sb.SuperbblasError, match="mask1"):
        sb.copy(1.0, p1, "ab", [0, 0], dim, dim, v1, p1, "ab", [0, 0], dim, v1, mask0=m1)


@pytest.mark.parametrize("t0,t1", [(np.float32, np.complex64), (np.float32, np.complex128),
                                   (np.float64, np.complex64), (np.float64, np.complex128)])
def test_copy_real_to_complex(gpu, t0, t1):
    import torch
    import superbblas_amd as sb
    dim0, dim1 = [5, 7, 3], [3, 5, 7]
    g = (np.arange(105) - 50).astype(t0)
    v0 = [torch.from_numpy(g).to(gpu)]
    v1 = [torch.from_numpy(np.full(105, 9 + 9j, t1)).to(gpu)]
    sb.copy(2.0, [([0, 0, 0], dim0)], "abc", [0, 0, 0], dim0, dim0, v0, [([0, 0, 0], dim1)],
            "cab", [0, 0, 0], dim1, v1)
    torch.cuda.synchronize()
    ref = (2.0 * g.reshape(dim0).transpose(2, 0, 1)).astype(t1).ravel()
    assert np.array_equal(v1[0].cpu().numpy(), ref)


def test_copy_fast_path_replay(gpu):
    """The C ABI's copy fast path (a launch tape recorded by the first call of a shape and
    replayed by later calls on other pointers): repeated calls of one shape with new buffers,
    other alphas, Copy/Add, multi-component operands and an in-place (aliased) copy all match the
    oracle bit-exactly."""
    import torch
    import superbblas_amd as sb
    dim0, dim1 = [4, 3, 5, 2], [5, 2, 4, 3]  # "abcd" -> "cdab"
    p0 = sb.basic_partitioning("abcd", dim0, [2, 1, 1, 1], "a", 2, 1)  # two components
    p1 = [([0, 0, 0, 0], dim1)]
    from0, size0, from1 = [1, 0, 2, 1], [3, 3, 4, 2], [1, 1, 2, 0]
    for rep, (alpha, add) in enumerate([(1.0, False), (2.0, False), (-0.5j, True), (1.0, True),
                                        (0.0, False), (3.0, False)]):
        g0 = int_valued(_vol(dim0), np.complex128, 10 + rep)
        g1 = int_valued(_vol(dim1), np.complex128, 20 + rep)
        ref = g1.copy()
        oracle_copy(alpha, "abcd", from0, size0, dim0, g0, "cdab", from1, dim1, ref, add=add)
        g0r = g0.reshape(dim0)
        v0 = [torch.from_numpy(np.ascontiguousarray(g0r[f[0]:f[0] + s[0]]).ravel()).to(gpu)
              for f, s in p0]
        v1 = torch.from_numpy(g1).to(gpu)
        sb.copy(alpha, p0, "abcd", from0, size0, dim0, v0, p1, "cdab", from1, dim1, [v1],
                copyadd=sb.Add if add else sb.Copy)
        torch.cuda.synchronize()
        assert np.array_equal(v1.cpu().numpy().view(np.uint8), ref.view(np.uint8)), rep
    # in place: shift a tensor onto itself twice (aliased origin / destination)
    dim = [6, 5]
    for rep in range(2):
        g = int_valued(30, np.complex128, 40 + rep)
        ref = g.copy()
        src = g.copy()
        oracle_copy(1.0, "ab", [0, 0], [3, 5], dim, src, "ab", [3, 0], dim, ref)
        t = torch.from_numpy(g).to(gpu)
        sb.copy(1.0, [([0, 0], dim)], "ab", [0, 0], [3, 5], dim, [t], [([0, 0], dim)], "ab",
                [3, 0], dim, [t])
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy().view(np.uint8), ref.view(np.uint8)), rep


@pytest.mark.parametrize("t0,t1", [(np.complex64, np.complex64), (np.float64, np.float64),
                                   (np.uint64, np.uint64), (np.complex64, np.complex128),
                                   (np.complex128, np.complex64), (np.float64, np.complex64)])
def test_paired_8byte_transposes(gpu, t0, t1):
    """The tiled kernel's paired (16-byte) accesses for 8-byte elements: the chain's n <-> c <->
    xyz redistribution (source chain first), its contraction-operand reorder, a whole-tensor
    permute; even and odd rhs counts (odd tile rows are rounded to even ones), boxes at odd
    origins (8-byte aligned pointers fall back), alpha and Add (paired reads only), and the
    single-access form (copy.pair -1) on the same shapes."""
    cases = [("tnsxyzc", "pxyztscn", lambda n: ([4, n, 4, 4, 4, 4, 3], [1, 4, 4, 4, 4, 4, 3, n])),
             ("pXYZTSCn", "TSnpXYZC", lambda n: ([1, 4, 4, 4, 4, 4, 3, n], [4, 4, n, 1, 4, 4, 4, 3])),
             ("xyztnsc", "tnsxyzc", lambda n: ([4, 4, 4, 4, n, 4, 3], [4, n, 4, 4, 4, 4, 3]))]
    import superbblas_amd as sb
    forms = set()

    def run(o0, o1, dims, n, shift, add):
        dim0, dim1 = dims(n)
        size0 = list(dim0)
        from0 = [0] * len(dim0)
        from1 = [0] * len(dim1)
        if shift:  # a box one short in the rhs dim, at rhs origin 1 on both sides
            i0, i1 = o0.index("n" if "n" in o0 else "N"), o1.index("n" if "n" in o1 else "N")
            size0[i0] -= 1
            from0[i0] = 1
            from1[i1] = 1
        kind = np.dtype(t0).kind
        v0 = index_valued(_vol(dim0), t0) if kind == "u" else int_valued(_vol(dim0), t0, 3)
        v1 = np.arange(_vol(dim1)).astype(t1) if np.dtype(t1).kind == "u" else \
            int_valued(_vol(dim1), t1, 4)
        alpha = 1.0 if kind == "u" else (2.0 - 1.0j if kind == "c" else 3.0)
        ref = v1.copy()
        oracle_copy(alpha, o0, from0, size0, dim0, v0, o1, from1, dim1, ref, add=add)
        out = _gpu_local_copy(gpu, alpha, o0, from0, size0, dim0, v0, o1, from1, dim1, v1.copy(),
                              add=add)
        forms.add(sb.tune_get("copy.last_pair"))
        assert np.array_equal(out.view(np.uint8), ref.view(np.uint8)), (o0, o1, n, shift, add)

    # the library's defaults (the transpose kernels take most of these shapes): bit-exact
    for (o0, o1, dims), n, shift, add in itertools.product(cases, (6, 5), (0, 1), (False, True)):
        if add and np.dtype(t1).kind == "u":
            continue
        run(o0, o1, dims, n, shift, add)
    # the tile kernel itself (transpose kernels off): paired and single-access forms
    forms.clear()
    sb.tune_set("copy.trans", -1)
    sb.tune_set("copy.btrans", -1)
    try:
        for (o0, o1, dims), n, shift, add in itertools.product(cases, (6, 5), (0, 1), (False, True)):
            if add and np.dtype(t1).kind == "u":
                continue
            run(o0, o1, dims, n, shift, add)
        # the single-access form on the same shapes (odd tile rows are rounded to even ones, so
        # the defaults above may pair every case)
        prev = sb.tune_get("copy.pair")
        sb.tune_set("copy.pair", -1)
        try:
            for (o0, o1, dims), n in itertools.product(cases, (6, 5)):
                run(o0, o1, dims, n, 0, False)
        finally:
            sb.tune_set("copy.pair", prev)
    finally:
        sb.tune_set("copy.trans", 0)
        sb.tune_set("copy.btrans", 0)
    # paired reads ran for 8-byte sources, paired writes for 8-byte destinations, and the
    # single-access fallback ran too
    assert 0 in forms, forms
    assert any(f & 1 for f in forms) == (np.dtype(t0).itemsize == 8), forms
    assert any(f & 2 for f in forms) == (np.dtype(t1).itemsize == 8), forms

