"""Ragged last workgroups of every LDS-DMA kernel (the overrun class fixed in 39cd2bc: a DMA pass
writes whole rows of 16-B lanes, so the last, partial chunk of a launch is where an undersized LDS
allocation or a pass past the data would show).  Each case picks a row count that is not a
multiple of the kernel's rows per workgroup, asserts the kernel form that ran, and compares with
the oracle exactly (integer-valued data).  The launchers also check their dynamic LDS against the
DMA passes of their kernel's loop (check_dma_lds, sbx_internal.h) and throw on a shortfall."""
import numpy as np
import pytest

from _common import T_CDOUBLE, TYPE_OF, oracle_bsr, oracle_kron_bsr, stencil_jj

pytestmark = pytest.mark.gpu


def _ints(rng, n, dtype):
    v = rng.integers(-4, 5, n) + (1j * rng.integers(-4, 5, n) if np.dtype(dtype).kind == "c" else 0)
    return v.astype(dtype)


@pytest.mark.parametrize("dims", [(3, 3, 3, 3), (3, 5, 4, 5), (1, 7, 1, 5)])
@pytest.mark.parametrize("ncols,form", [(1, 1), (2, 1), (3, 1), (5, 2), (12, 2), (29, 2),
                                        (40, 3), (64, 3)])
def test_3x3_tails(gpu, dims, ncols, form):
    """bsr_ell9_row_kernel (28 rows / workgroup), bsr_ell9_split_kernel (rows by the thread and
    LDS budgets), bsr_ell9_kernel (row chunks by 12 KB of values): ragged row counts 81, 300, 35"""
    import torch
    import superbblas_amd as sb
    rng = np.random.default_rng(ncols)
    dt = np.complex128
    vol = int(np.prod(dims))
    jj = stencil_jj(dims).reshape(-1)
    ii = np.full(vol, 9, np.int32)
    vals = _ints(rng, vol * 81, dt)
    x = _ints(rng, vol * 3 * ncols, dt)
    dim = list(dims) + [1, 3]
    yref = np.zeros(vol * 3 * ncols, dt)
    oracle_bsr(T_CDOUBLE, dim, 0, vol, 3, 3, ii, jj, vals, False, x, ncols, True, yref, ncols,
               True, ncols, 1.0)
    full = [([0] * 6, dim)]
    op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                       [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                       [torch.from_numpy(vals).to(gpu)])
    dimx = [1] + list(dims) + [1, 3, ncols]
    ty = torch.full((vol * 3 * ncols,), 5.0, dtype=torch.complex128, device=gpu)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTSCn", [0] * 8, dimx, dimx,
                  [torch.from_numpy(x).to(gpu)], 0.0, [([0] * 8, dimx)], "pxyztscn", [0] * 8,
                  dimx, dimx, "p", [ty])
    torch.cuda.synchronize()
    used = sb.tune_get("bsr.last_kernel")
    op.destroy()
    assert used == form, used
    assert np.array_equal(ty.cpu().numpy(), yref)


@pytest.mark.parametrize("dtype,ncols,form", [(np.complex128, 12, 7), (np.complex128, 5, 7),
                                              (np.complex64, 12, 8), (np.complex64, 16, 8),
                                              (np.complex64, 7, 7), (np.float64, 12, 8)])
def test_12x12_tails(gpu, dtype, ncols, form):
    """bsr_mfma_dma_kernel (4 rows per workgroup, one ring of 2 slots per wave; packed slots for
    8-byte elements) on 81 block rows"""
    import torch
    import superbblas_amd as sb
    rng = np.random.default_rng(ncols)
    dims = (3, 3, 3, 3)
    vol, b = 81, 12
    jj = stencil_jj(dims).reshape(-1)
    ii = np.full(vol, 9, np.int32)
    vals = _ints(rng, vol * 9 * b * b, dtype)
    x = _ints(rng, vol * b * ncols, dtype)
    dim = list(dims) + [4, 3]
    yref = np.zeros(vol * b * ncols, dtype)
    oracle_bsr(TYPE_OF[np.dtype(dtype)], dim, 0, vol, b, b, ii, jj, vals, False, x, ncols, True,
               yref, ncols, True, ncols, 1.0)
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, 4, 3]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, False, [torch.from_numpy(ii).to(gpu)],
                       [torch.from_numpy(jj).to(gpu)], [torch.from_numpy(vals).to(gpu)])
    dimx = [1] + list(dims) + [4, 3, ncols]
    ty = torch.zeros(vol * b * ncols, dtype=getattr(torch, np.dtype(dtype).name), device=gpu)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTSCn", [0] * 8, dimx, dimx,
                  [torch.from_numpy(x).to(gpu)], 0.0, [([0] * 8, dimx)], "pxyztscn", [0] * 8,
                  dimx, dimx, "p", [ty])
    torch.cuda.synchronize()
    used = sb.tune_get("bsr.last_kernel")
    op.destroy()
    assert used == form, used
    assert np.array_equal(ty.cpu().numpy(), yref)


@pytest.mark.parametrize("ncols,form,spin_first", [(8, 6, 0), (12, 6, 0), (16, 5, 0), (20, 5, 0),
                                                    (8, 9, 1), (12, 9, 1), (20, 9, 1)])
def test_kron_tails(gpu, ncols, form, spin_first):
    """bsr_kron_mfma_packed_kernel (rw = 16 W / n rows per workgroup), bsr_kron_mfma_kernel (4
    (row, column group) tasks per workgroup) and bsr_kron_spin_kernel (64 (row, column) pairs per
    wave, rows in the XCD order) on a 3^4 lattice: 81 block rows"""
    import torch
    import superbblas_amd as sb
    rng = np.random.default_rng(ncols)
    L, spin, color = 3, 4, 3
    dims = (L, L, L, L)
    V = L ** 4
    jj = stencil_jj(dims).reshape(-1)
    ii = np.full(V, 9, np.int32)
    vals = _ints(rng, V * 9 * color * color, np.complex128)
    kron = _ints(rng, 9 * spin * spin, np.complex128)
    if spin_first:  # two nonzeros per spin row (the spin-first kernel's shape)
        kron = kron.reshape(9, 4, 4)
        kron[:, :, 1:3] = 0
        kron = kron.ravel().copy()
    x = _ints(rng, V * color * ncols * spin, np.complex128)
    yref = np.zeros_like(x)
    oracle_kron_bsr(T_CDOUBLE, [L, L, L, L, 1, 1], 0, V, 9, color, color, spin, spin, jj, vals,
                    kron, False, x, yref, ncols, 1.0)
    dim = [L, L, L, L, spin, color]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, False,
                            [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                            [torch.from_numpy(vals).to(gpu)], [torch.from_numpy(kron).to(gpu)])
    dimx = [1, L, L, L, L, color, ncols, spin]
    ty = torch.zeros(len(x), dtype=torch.complex128, device=gpu)
    sb.tune_set("bsr.kron_spin", spin_first)
    try:
        sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTCnS", [0] * 8, dimx,
                      dimx, [torch.from_numpy(x).to(gpu)], 0.0, [([0] * 8, dimx)], "pxyztcns",
                      [0] * 8, dimx, dimx, "p", [ty])
        torch.cuda.synchronize()
        used = sb.tune_get("bsr.last_kernel")
    finally:
        sb.tune_set("bsr.kron_spin", 0)
        op.destroy()
    assert used == form, used
    assert np.array_equal(ty.cpu().numpy(), yref)


@pytest.mark.parametrize("dtype,m,n,k,batch", [(np.complex128, 129, 131, 300, 2),
                                               (np.complex128, 256, 256, 1000, 1),
                                               (np.complex64, 47, 45, 777, 5),
                                               (np.float64, 130, 70, 96, 3)])
def test_gemm_dma_tails(gpu, dtype, m, n, k, batch):
    """gemm_dma_kernel (128x128 and 48x48 tiles, static LDS sized to its DMA lanes by
    static_assert): partial last tiles in M and N, a partial last K slab; integer data, exact"""
    import torch
    import superbblas_amd as sb
    rng = np.random.default_rng(m)
    tt = getattr(torch, np.dtype(dtype).name)
    a = torch.from_numpy(_ints(rng, k * m * batch, dtype)).to(gpu)
    b = torch.from_numpy(_ints(rng, k * n * batch, dtype)).to(gpu)
    c = torch.zeros(m * n * batch, dtype=tt, device=gpu)
    # C (m x n, column-major) = A^T B with A stored k x m, B k x n (the contraction's 'T','N')
    sb.xgemm_batch_strided("T", "N", m, n, k, 1.0, a, k, k * m, b, k, k * n, 0.0, c, m, m * n,
                           batch)
    torch.cuda.synchronize()
    A = a.cpu().numpy().reshape(batch, m, k).astype(np.complex128)
    B = b.cpu().numpy().reshape(batch, n, k).astype(np.complex128)
    ref = np.einsum("bmk,bnk->bnm", A, B).reshape(-1)
    assert np.array_equal(c.cpu().numpy().astype(np.complex128), ref)
