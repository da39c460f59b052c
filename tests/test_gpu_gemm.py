"""Batched GEMM kernel (MFMA) vs the oracle's column-major batched GEMM
(blas_cpu_tmpl.hpp:405-477 restated in oracle/oracle.c).  Tolerance: 1e-10 relative
(Frobenius) for f64/complex<f64> (north_star), 1e-5 for f32/complex<f32>."""
import numpy as np
import pytest

from _common import oracle_gemm, random_valued, rel_err

pytestmark = pytest.mark.gpu

TOL = {np.complex128: 1e-10, np.float64: 1e-10, np.complex64: 1e-5, np.float32: 1e-5}


def _run(gpu, dtype, ta, tb, m, n, k, batch, alpha, beta, pad=0):
    import torch
    import superbblas_amd as sb
    lda = (m if ta == "N" else k) + pad
    ldb = (k if tb == "N" else n) + pad
    ldc = m + pad
    sa = lda * (k if ta == "N" else m) + pad
    sb_ = ldb * (n if tb == "N" else k) + pad
    sc = ldc * n + pad
    a = random_valued(sa * batch, dtype, 1)
    b = random_valued(sb_ * batch, dtype, 2)
    c = random_valued(sc * batch, dtype, 3)
    ref = c.copy()
    oracle_gemm(ta, tb, m, n, k, alpha, a, lda, sa, b, ldb, sb_, beta, ref, ldc, sc, batch)
    ta_, tb_, tc_ = (torch.from_numpy(x).to(gpu) for x in (a, b, c))
    sb.xgemm_batch_strided(ta, tb, m, n, k, alpha, ta_, lda, sa, tb_, ldb, sb_, beta, tc_, ldc,
                           sc, batch)
    torch.cuda.synchronize()
    out = tc_.cpu().numpy()
    return out, ref


@pytest.mark.parametrize("dtype", [np.complex128, np.float64, np.complex64, np.float32])
@pytest.mark.parametrize("ta,tb", [(x, y) for x in "NTC" for y in "NTC"])
def test_gemm_small(gpu, dtype, ta, tb):
    out, ref = _run(gpu, dtype, ta, tb, 37, 21, 45, 3, 1.5 - 0.5j, 0.25 + 1j, pad=3)
    assert rel_err(out, ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [np.complex128, np.float64])
def test_gemm_lattice_shape(gpu, dtype):
    # the config-2 GEMM shape scaled down: ('T','N', m = n = 64, k = 1536, batch = 8)
    out, ref = _run(gpu, dtype, "T", "N", 64, 64, 1536, 8, 1.0, 0.0)
    assert rel_err(out, ref) < TOL[dtype]


@pytest.mark.parametrize("m,n,k,batch", [(1, 1, 1, 1), (1, 7, 300, 2), (65, 1, 17, 3),
                                         (130, 66, 5, 1), (16, 16, 4000, 2)])
def test_gemm_edges(gpu, m, n, k, batch):
    out, ref = _run(gpu, np.complex128, "T", "N", m, n, k, batch, 1.0, -1.0)
    assert rel_err(out, ref) < 1e-10


def test_gemm_k0_and_alpha0(gpu):
    out, ref = _run(gpu, np.complex128, "N", "N", 8, 8, 0, 2, 1.0, 2.0)
    assert rel_err(out, ref) < 1e-14
    out, ref = _run(gpu, np.complex128, "N", "N", 8, 8, 8, 2, 0.0, 0.0)
    assert np.all(out == 0)


def test_gemm_beta0_ignores_nan(gpu):
    """beta == 0 overwrites C (tensor.h:1511-1512): NaNs in C must not propagate."""
    import torch
    import superbblas_amd as sb
    a = torch.ones(16 * 16, dtype=torch.complex128, device=gpu)
    b = torch.ones(16 * 16, dtype=torch.complex128, device=gpu)
    c = torch.full((16 * 16,), float("nan"), dtype=torch.complex128, device=gpu)
    sb.xgemm_batch_strided("N", "N", 16, 16, 16, 1.0, a, 16, 0, b, 16, 0, 0.0, c, 16, 0, 1)
    torch.cuda.synchronize()
    assert torch.all(c == 16)


@pytest.mark.parametrize("dtype", [np.complex128, np.float64, np.complex64, np.float32])
@pytest.mark.parametrize("ta,tb", [("T", "N"), ("N", "N"), ("N", "T"), ("C", "N"), ("T", "C")])
@pytest.mark.parametrize("m,n,k", [(96, 80, 128), (256, 192, 512)])
def test_gemm_granule_shapes(gpu, dtype, ta, tb, m, n, k):
    # extents that are multiples of the 16-byte granule of every type: the LDS-DMA kernel path
    out, ref = _run(gpu, dtype, ta, tb, m, n, k, 3, 0.5 + 1j, -0.75)
    assert rel_err(out, ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [np.complex128, np.float64, np.complex64, np.float32])
@pytest.mark.parametrize("ta,tb", [("T", "N"), ("N", "N"), ("N", "T"), ("C", "N"), ("T", "C")])
@pytest.mark.parametrize("m,n,k,batch", [(48, 48, 768, 3), (34, 46, 520, 2), (48, 40, 4096, 1)])
@pytest.mark.parametrize("t48", [1, 2, 3, 4, 5, 6])
def test_gemm_48_tiles(gpu, dtype, ta, tb, m, n, k, batch, t48):
    """33..48 rows and columns: the 48x48 LDS-DMA tile forms (sbx_tune_set "gemm.t48"; the
    chain's TSnsN contraction shape), with split-K over the long k; 5 = the library's choice, 6
    = four k-groups of the whole tile per workgroup"""
    import superbblas_amd as sb
    old = sb.tune_get("gemm.t48")
    sb.tune_set("gemm.t48", t48)
    try:
        out, ref = _run(gpu, dtype, ta, tb, m, n, k, batch, 0.5 + 1j, -1.0)
    finally:
        sb.tune_set("gemm.t48", old)
    assert rel_err(out, ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [np.complex128, np.complex64, np.float64])
@pytest.mark.parametrize("m,k", [(256, 1536), (48, 3072), (300, 200)])
def test_gemm_same_operand(gpu, dtype, m, k):
    """A^H A (one buffer passed as both operands, 'C','N'): the workgroups on diagonal tiles stage
    one slab image for both operands (gemm.share_ab); off-diagonal tiles, the unshared form and the
    oracle agree -- bit-identically between the two forms."""
    import torch
    import superbblas_amd as sb
    batch = 3
    a = random_valued(k * m * batch, dtype, 5)
    ta = torch.from_numpy(a).to(gpu)
    outs = []
    for share in (1, 0):
        sb.tune_set("gemm.share_ab", share)
        c = torch.zeros(m * m * batch, dtype=ta.dtype, device=gpu)
        sb.xgemm_batch_strided("C" if np.dtype(dtype).kind == "c" else "T", "N", m, m, k, 1.0, ta,
                               k, k * m, ta, k, k * m, 0.0, c, m, m * m, batch)
        torch.cuda.synchronize()
        outs.append(c.cpu().numpy())
    sb.tune_set("gemm.share_ab", 1)
    ref = np.zeros(m * m * batch, dtype)
    oracle_gemm("C" if np.dtype(dtype).kind == "c" else "T", "N", m, m, k, 1.0, a, k, k * m, a, k,
                k * m, 0.0, ref, m, m * m, batch)
    assert np.array_equal(outs[0], outs[1])
    assert rel_err(outs[0], ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [np.complex128, np.complex64, np.float64])
@pytest.mark.parametrize("m,k,batch", [(48, 3072, 3), (40, 1000, 2), (48, 96, 5), (36, 24, 1)])
@pytest.mark.parametrize("tb", ["T", "C"])
@pytest.mark.parametrize("t48", [5, 13, 14, 16, 17])
def test_gemm_same_operand_mmajor(gpu, dtype, m, k, batch, tb, t48):
    """A op(A) with one M-major buffer as both operands and one output tile per batch entry (the
    chain's y^H y shape): the wave-private slab-ring kernel (A-only slab images, no barrier in the
    main loop; partial k ranges summed through LDS), against the oracle and the unshared form
    (within rounding: the k order of the two forms differs), with ragged k and m < 48"""
    import torch
    import superbblas_amd as sb
    if tb == "C" and np.dtype(dtype).kind != "c":
        tb = "T"
    a = random_valued(k * m * batch, dtype, 7)
    ta = torch.from_numpy(a).to(gpu)
    outs = []
    old = sb.tune_get("gemm.t48")
    sb.tune_set("gemm.t48", t48)
    try:
        for share in (1, 0):
            sb.tune_set("gemm.share_ab", share)
            c = torch.zeros(m * m * batch, dtype=ta.dtype, device=gpu)
            sb.xgemm_batch_strided("N", tb, m, m, k, 0.5 - 0.5j if np.dtype(dtype).kind == "c"
                                   else 0.5, ta, m, k * m, ta, m, k * m, 0.0, c, m, m * m, batch)
            torch.cuda.synchronize()
            outs.append(c.cpu().numpy())
    finally:
        sb.tune_set("gemm.share_ab", 1)
        sb.tune_set("gemm.t48", old)
    ref = np.zeros(m * m * batch, dtype)
    oracle_gemm("N", tb, m, m, k, 0.5 - 0.5j if np.dtype(dtype).kind == "c" else 0.5, a, m, k * m,
                a, m, k * m, 0.0, ref, m, m * m, batch)
    assert rel_err(outs[0], ref) < TOL[dtype]
    assert rel_err(outs[1], ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [np.complex128, np.complex64, np.float64])
@pytest.mark.parametrize("m,k,batch", [(48, 6144, 8), (40, 3000, 3), (48, 12288, 64)])
def test_gemm_fused_splitk_sum(gpu, dtype, m, k, batch):
    """gemm.t48 17: the wave-ring kernel with its split-K sum fused (write-through partials, the
    last workgroup of a batch entry sums the splits in split order and resets its counter):
    bit-identical to the two-kernel form (t48 5: the same partials, the same order), over
    repeated calls (the per-stream counters return to zero) and with beta != 0 (C read back)"""
    import torch
    import superbblas_amd as sb
    a = random_valued(k * m * batch, dtype, 11)
    ta = torch.from_numpy(a).to(gpu)
    c0 = random_valued(m * m * batch, dtype, 12)
    cplx = np.dtype(dtype).kind == "c"
    alpha, beta = (0.5 - 0.5j, 0.25 + 1j) if cplx else (0.5, 0.25)
    old = sb.tune_get("gemm.t48")
    outs = {}
    try:
        for t48 in (5, 17, 17, 17):
            sb.tune_set("gemm.t48", t48)
            c = torch.from_numpy(c0.copy()).to(gpu)
            sb.xgemm_batch_strided("N", "C" if cplx else "T", m, m, k, alpha, ta, m, k * m, ta, m,
                                   k * m, beta, c, m, m * m, batch)
            torch.cuda.synchronize()
            outs.setdefault(t48, []).append(c.cpu().numpy())
    finally:
        sb.tune_set("gemm.t48", old)
    for o in outs[17]:
        assert np.array_equal(o, outs[5][0])
    if batch > 8:  # (the chain's own shape: bit identity with the two-kernel form is the check)
        return
    ref = c0 * beta
    oracle_gemm("N", "C" if cplx else "T", m, m, k, alpha, a, m, k * m, a, m, k * m, 1.0, ref, m,
                m * m, batch)
    assert rel_err(outs[17][0], ref) < TOL[dtype]


# the skinny forms (blas.h:686-800's dot / gemv shortcuts; tests/dist.cpp:160-195's inner-product
# m = n <= 12, k = 6144 and update m = 6144, n = k <= 12 shapes): gemm_dot_kernel for m, n <= 4,
# gemm_rows_kernel for one dimension <= 16 and a short k (vectors with a long k: the MFMA tiles), the transposed problem
# for a short m; the same shapes through the MFMA tiles (gemm.skinny 0) agree with the oracle too
SKINNY = [(1, 1, 6144, 8), (2, 2, 6144, 8), (3, 4, 6000, 2), (4, 1, 100, 5), (1, 3, 7, 3),
          (6144, 1, 1, 8), (6144, 3, 3, 2), (1000, 12, 12, 2), (999, 16, 5, 1), (1, 700, 9, 2),
          (12, 500, 12, 2), (777, 1, 300, 2), (1, 500, 301, 1), (16, 1, 1 << 16, 1)]


@pytest.mark.parametrize("dtype", [np.complex128, np.float64, np.complex64, np.float32])
@pytest.mark.parametrize("ta,tb", [("N", "N"), ("T", "N"), ("C", "T"), ("N", "C"), ("T", "C")])
@pytest.mark.parametrize("m,n,k,batch", SKINNY)
@pytest.mark.parametrize("skinny", [1, 0])
def test_gemm_skinny(gpu, dtype, ta, tb, m, n, k, batch, skinny):
    import superbblas_amd as sb
    old = sb.tune_get("gemm.skinny")
    sb.tune_set("gemm.skinny", skinny)
    try:
        out, ref = _run(gpu, dtype, ta, tb, m, n, k, batch, 0.5 + 0.25j, -1.0 + 0.5j, pad=1)
    finally:
        sb.tune_set("gemm.skinny", old)
    assert rel_err(out, ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [np.complex128, np.float64, np.complex64])
@pytest.mark.parametrize("m,n,k,batch", [(256, 256, 1000, 2), (129, 200, 16, 1), (300, 140, 40, 3),
                                         (128, 128, 8, 1)])
def test_gemm_loader_forms(gpu, dtype, m, n, k, batch):
    """the slab DMA by 8 loader waves, spread over 1 / 4 k-steps or with the early barrier
    (gemm.dma_spread 0: a slab's barrier before its last k-step), and by every wave (loaders
    0): against the oracle and bit-identical to one another (the same MFMA order); partial
    tiles and partial, single and half slabs"""
    import torch
    import superbblas_amd as sb
    old_l, old_s = sb.tune_get("gemm.loaders"), sb.tune_get("gemm.dma_spread")
    outs = []
    try:
        for lw, sp in ((8, 1), (8, 0), (8, 4), (0, 1)):
            sb.tune_set("gemm.loaders", lw)
            sb.tune_set("gemm.dma_spread", sp)
            out, ref = _run(gpu, dtype, "T", "N", m, n, k, batch, 1.0, 0.0)
            assert rel_err(out, ref) < TOL[dtype], (lw, sp)
            outs.append(out)
    finally:
        sb.tune_set("gemm.loaders", old_l)
        sb.tune_set("gemm.dma_spread", old_s)
    for o in outs[1:3]:
        assert np.array_equal(o, outs[0])


def test_host_context_calls_use_current_device(gpu):
    """detail::xgemm_batch_strided and copy_n on host (CPU-context) operands run on the calling
    thread's current device (the reference's CPU path runs on the calling rank, platform.h:757-816),
    not on device 0: the device used is read back through the "detail.last_device" tune key"""
    import ctypes
    import torch
    import superbblas_amd as sb
    lib, ctx = sb._lib, sb._Ctx
    dev = torch.cuda.current_device()
    m, n, k = 5, 3, 7
    a = random_valued(m * k, np.complex128, 1)
    b = random_valued(k * n, np.complex128, 2)
    c = np.zeros(m * n, np.complex128)
    ref = c.copy()
    oracle_gemm("N", "N", m, n, k, 1.0, a, m, 0, b, k, 0, 0.0, ref, m, 0, 1)
    one, zero = (ctypes.c_double * 2)(1.0, 0.0), (ctypes.c_double * 2)(0.0, 0.0)
    vp = ctypes.c_void_p
    rc = lib.sbx_xgemm_batch_strided_ctx(
        3, ctypes.c_char(b"N"), ctypes.c_char(b"N"), m, n, k, one, vp(a.ctypes.data), m,
        ctypes.c_longlong(0), vp(b.ctypes.data), k, ctypes.c_longlong(0), zero, vp(c.ctypes.data), m,
        ctypes.c_longlong(0), 1, ctx(sb.CPU, -1))
    assert rc == 0, sb._lib.sbx_last_error()
    assert rel_err(c, ref) < 1e-12
    assert sb.tune_get("detail.last_device") == dev
    # copy_n between host buffers (through device scratch): the same device
    src = np.arange(16, dtype=np.float64)
    dst = np.zeros(16, np.float64)
    rc = lib.sbx_copy_n_blocking(one, 1, vp(src.ctypes.data), ctx(sb.CPU, -1), ctypes.c_longlong(1),
                                 None, ctx(sb.CPU, -1), ctypes.c_longlong(16), 1, vp(dst.ctypes.data),
                                 ctx(sb.CPU, -1), None, ctx(sb.CPU, -1), 0)
    assert rc == 0, sb._lib.sbx_last_error()
    assert np.array_equal(dst, src)
    assert sb.tune_get("detail.last_device") == dev


# tests/dist.cpp's xgemm_batch_strided sweep at a reduced k (inner products m = n, k = volume;
# updates m = volume, n = k) and neighbouring shapes: gemm_frag_kernel (MFMA fragments straight
# from global memory; gemm.frag 1, the default) against the oracle, with partial tiles, split-K
# and every trans pair; gemm.frag 0 runs the same shapes through the other kernels
FRAG = [(5, 5, 6144, 4), (8, 8, 6144, 4), (12, 12, 3000, 3), (16, 16, 6144, 2), (32, 32, 4096, 2),
        (17, 30, 777, 3), (6144, 8, 8, 2), (6144, 12, 12, 2), (3000, 16, 16, 1), (999, 13, 64, 2),
        (16, 1, 1 << 15, 1), (1, 16, 1 << 15, 1), (16, 5000, 7, 1), (1000, 3, 50, 2),
        # tall-skinny with a short dimension of 17-48 (the fragment kernel for complex<float>)
        (4100, 32, 32, 2), (24, 3001, 20, 2), (2050, 17, 64, 1), (3000, 48, 48, 1)]


@pytest.mark.parametrize("dtype", [np.complex128, np.float64, np.complex64, np.float32])
@pytest.mark.parametrize("ta,tb", [("N", "N"), ("T", "N"), ("C", "N"), ("N", "C"), ("C", "T")])
@pytest.mark.parametrize("m,n,k,batch", FRAG)
@pytest.mark.parametrize("frag", [1, 0])
def test_gemm_frag(gpu, dtype, ta, tb, m, n, k, batch, frag):
    import superbblas_amd as sb
    old = sb.tune_get("gemm.frag")
    sb.tune_set("gemm.frag", frag)
    try:
        out, ref = _run(gpu, dtype, ta, tb, m, n, k, batch, 0.5 - 0.25j, 0.75 + 0.5j, pad=1)
    finally:
        sb.tune_set("gemm.frag", old)
    assert rel_err(out, ref) < TOL[dtype]


FRAG_PAIRS = [(12, 12, 4096, 3), (32, 32, 2048, 2), (5, 9, 1000, 2), (4100, 32, 32, 2),
              (2050, 24, 64, 1), (8, 8, 1001, 2)]


@pytest.mark.parametrize("dtype", [np.complex64, np.float64])
@pytest.mark.parametrize("ta,tb", [("T", "N"), ("C", "N"), ("N", "N"), ("C", "T")])
@pytest.mark.parametrize("m,n,k,batch", FRAG_PAIRS)
@pytest.mark.parametrize("pad", [0, 2])
@pytest.mark.parametrize("pair", [1, 0])
def test_gemm_frag_pairs(gpu, dtype, ta, tb, m, n, k, batch, pad, pair):
    """gemm_frag_kernel with 8-byte elements: an operand with unit k stride and even strides reads
    its k pairs as one 16-byte load (gemm.frag_pair; the pair permutes a load group's k the same
    way for A and B), odd k or odd strides keep the element loads"""
    import superbblas_amd as sb
    old = sb.tune_get("gemm.frag_pair")
    sb.tune_set("gemm.frag_pair", pair)
    try:
        out, ref = _run(gpu, dtype, ta, tb, m, n, k, batch, 0.5 - 0.25j, 0.75 + 0.5j, pad=pad)
    finally:
        sb.tune_set("gemm.frag_pair", old)
    assert rel_err(out, ref) < TOL[dtype]


FRAG_NT = [(4100, 64, 64, 2), (2050, 48, 32, 1), (999, 40, 17, 2), (32, 32, 4096, 2),
           (12, 12, 3000, 3), (6144, 8, 8, 2)]


@pytest.mark.parametrize("dtype", [np.complex128, np.float64, np.complex64, np.float32])
@pytest.mark.parametrize("ta,tb", [("N", "N"), ("C", "N"), ("N", "T")])
@pytest.mark.parametrize("m,n,k,batch", FRAG_NT)
@pytest.mark.parametrize("nt", [2, 4])
def test_gemm_frag_nt(gpu, dtype, ta, tb, m, n, k, batch, nt):
    """gemm_frag_kernel with NT 16 x 16 tiles per wave along n (gemm.frag_nt; the A fragments
    loaded once for the NT tiles), the tall form widened to 64 columns (gemm.frag_tall)"""
    import superbblas_amd as sb
    old_nt, old_tall = sb.tune_get("gemm.frag_nt"), sb.tune_get("gemm.frag_tall")
    sb.tune_set("gemm.frag_nt", nt)
    sb.tune_set("gemm.frag_tall", 64)
    try:
        out, ref = _run(gpu, dtype, ta, tb, m, n, k, batch, 0.5 - 0.25j, 0.75 + 0.5j, pad=1)
    finally:
        sb.tune_set("gemm.frag_nt", old_nt)
        sb.tune_set("gemm.frag_tall", old_tall)
    assert rel_err(out, ref) < TOL[dtype]
