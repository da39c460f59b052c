"""bsr_krylov on the GPU vs the oracle's builtin BSR loop (bsr.h:535-650), on the 9-point
lattice stencil of tests/bsr.cpp:169-255 with its integer-valued nonzeros (exact)."""
import numpy as np
import pytest

from _common import T_CDOUBLE, oracle_bsr, rel_err

pytestmark = pytest.mark.gpu


def lattice_operator(L, spin, color, dtype=np.complex128):
    """9-point periodic stencil on an L^4 lattice, blocks (spin*color)^2, image = domain =
    xyztsc; jj coordinates relative to the (whole) domain (bsr.cpp:169-255)."""
    dim = [L, L, L, L, spin, color]
    vol = L ** 4
    b = spin * color
    sites = np.array(np.unravel_index(np.arange(vol), (L, L, L, L))).T
    jj, nb = [], 0
    for s in sites:
        nbrs = [s.copy()]
        for d in range(4):
            if L == 1:
                continue
            for dr in (-1, 1):
                c = s.copy()
                c[d] = (c[d] + dr) % L
                nbrs.append(c)
                if L <= 2:
                    break
        nb = len(nbrs)
        for c in nbrs:
            jj.append(list(c) + [0, 0])
    jj = np.array(jj, dtype=np.int32)
    ii = np.full(vol, nb, dtype=np.int32)
    nnz = vol * nb
    k = np.arange(nnz * b * b, dtype=np.int64)
    vals = ((k * 3 + 1) % 7 - 3) + 1j * ((k * 5 + 2) % 9 - 4)
    if np.dtype(dtype).kind != "c":
        vals = vals.real
    return dim, ii, jj, vals.astype(dtype), nb


@pytest.mark.parametrize("spin,color,ncols", [(1, 3, 1), (1, 3, 5), (4, 3, 2), (1, 3, 600)])
@pytest.mark.parametrize("y_layout", ["row", "col"])
def test_bsr_lattice(gpu, spin, color, ncols, y_layout):
    """(600 rhs columns: past the row-chunk kernel's 512, the generic ELL kernel)"""
    import torch
    import superbblas_amd as sb
    L = 4
    dim, ii, jj, vals, nb = lattice_operator(L, spin, color)
    b = spin * color
    vol = L ** 4
    x = (np.arange(vol * b * ncols) % 17 - 8 + 1j * (np.arange(vol * b * ncols) % 5)).astype(
        np.complex128)
    # x: pXYZTSCn (row major, n fastest)
    yref = np.zeros(vol * b * ncols, np.complex128)
    oracle_bsr(T_CDOUBLE, dim, 0, vol, b, b, ii, jj, vals, False, x, ncols, True, yref,
               ncols if y_layout == "row" else vol * b, y_layout == "row", ncols, 1.0)
    full = [([0] * 6, dim)]
    op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, spin, color], [1, 1, 1, 1, spin, color],
                       False, [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                       [torch.from_numpy(vals).to(gpu)])
    dimx = [1, L, L, L, L, spin, color, ncols]
    tx = torch.from_numpy(x).to(gpu)
    if y_layout == "row":
        oy, dimy = "pxyztscn", [1, L, L, L, L, spin, color, ncols]
    else:
        oy, dimy = "pnxyztsc", [1, ncols, L, L, L, L, spin, color]
    ty = torch.zeros(vol * b * ncols, dtype=torch.complex128, device=gpu)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTSCn", [0] * 8, dimx, dimx,
                  [tx], 0.0, [([0] * 8, dimy)], oy, [0] * 8, dimy, dimy, "p", [ty])
    torch.cuda.synchronize()
    assert rel_err(ty.cpu().numpy(), yref) == 0.0
    op.destroy()


@pytest.mark.parametrize("spin,color,ncols", [(1, 3, 3), (4, 3, 2), (4, 3, 17)])
@pytest.mark.parametrize("variant", [0, 1])
def test_bsr_ragged_rows(gpu, spin, color, ncols, variant):
    """Rows with 0..9 nonzero blocks (a CSR operator, not ELL): the general-row kernels (12x12:
    the one-block-ahead MFMA kernel, variant 0, and the generic-row kernels, variant 1), exact."""
    import torch
    import superbblas_amd as sb
    L = 4
    dim, ii, jj, vals, nb = lattice_operator(L, spin, color)
    b = spin * color
    vol = L ** 4
    keep = np.arange(vol) % (nb + 1)  # row r keeps its first r % 10 blocks
    sel = np.concatenate([np.arange(r * nb, r * nb + keep[r]) for r in range(vol)])
    ii2 = keep.astype(np.int32)
    jj2 = jj.reshape(vol * nb, 6)[sel].reshape(-1).astype(np.int32)
    vals2 = vals.reshape(vol * nb, b * b)[sel].reshape(-1)
    x = (np.arange(vol * b * ncols) % 13 - 6 + 1j * (np.arange(vol * b * ncols) % 3)).astype(
        np.complex128)
    yref = np.zeros(vol * b * ncols, np.complex128)
    oracle_bsr(T_CDOUBLE, dim, 0, vol, b, b, ii2, jj2, vals2, False, x, ncols, True, yref, ncols,
               True, ncols, 1.0)
    full = [([0] * 6, dim)]
    sb.tune_set("bsr.variant", variant)
    try:
        op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, spin, color],
                           [1, 1, 1, 1, spin, color], False, [torch.from_numpy(ii2).to(gpu)],
                           [torch.from_numpy(jj2).to(gpu)], [torch.from_numpy(vals2).to(gpu)])
        dimx = [1, L, L, L, L, spin, color, ncols]
        ty = torch.full((vol * b * ncols,), 7.0, dtype=torch.complex128, device=gpu)
        sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTSCn", [0] * 8, dimx,
                      dimx, [torch.from_numpy(x).to(gpu)], 0.0, [([0] * 8, dimx)], "pxyztscn",
                      [0] * 8, dimx, dimx, "p", [ty])
        torch.cuda.synchronize()
        op.destroy()
    finally:
        sb.tune_set("bsr.variant", 0)
    assert np.array_equal(ty.cpu().numpy(), yref)


@pytest.mark.parametrize("dtype,ttype", [(np.complex64, 2), (np.float64, 1), (np.float32, 0)])
@pytest.mark.parametrize("spin,color,ncols", [(1, 3, 5), (4, 3, 3), (4, 3, 20)])
def test_bsr_lattice_types(gpu, dtype, ttype, spin, color, ncols):
    """Other element types on the 3x3 (ELL) and 12x12 (MFMA) kernels, x/y row major; small
    integer values so every type is exact."""
    import torch
    import superbblas_amd as sb
    L = 4
    dim, ii, jj, vals, nb = lattice_operator(L, spin, color)
    vals = (vals.real if np.dtype(dtype).kind == "f" else vals).astype(dtype)
    b = spin * color
    vol = L ** 4
    g = np.arange(vol * b * ncols)
    x = ((g % 7 - 3) + (1j * (g % 5 - 2) if np.dtype(dtype).kind == "c" else 0)).astype(dtype)
    yref = np.zeros(vol * b * ncols, dtype)
    oracle_bsr(ttype, dim, 0, vol, b, b, ii, jj, vals, False, x, ncols, True, yref, ncols, True,
               ncols, 1.0)
    full = [([0] * 6, dim)]
    op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, spin, color], [1, 1, 1, 1, spin, color],
                       False, [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                       [torch.from_numpy(vals).to(gpu)])
    dimx = [1, L, L, L, L, spin, color, ncols]
    ty = torch.zeros(vol * b * ncols, dtype=torch.from_numpy(x).dtype, device=gpu)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTSCn", [0] * 8, dimx, dimx,
                  [torch.from_numpy(x).to(gpu)], 0.0, [([0] * 8, dimx)], "pxyztscn", [0] * 8,
                  dimx, dimx, "p", [ty])
    torch.cuda.synchronize()
    assert np.array_equal(ty.cpu().numpy(), yref)
    op.destroy()


@pytest.mark.parametrize("spin,color,ncols,power", [(1, 3, 2, 3), (4, 3, 3, 2)])
def test_bsr_powers(gpu, spin, color, ncols, power):
    """okr powers (bsr.h:2211-2247): y[.., p, ..] = alpha A^(p+1) x + beta y[.., p, ..]."""
    import torch
    import superbblas_amd as sb
    L = 4
    dim, ii, jj, vals, nb = lattice_operator(L, spin, color)
    b = spin * color
    vol = L ** 4
    g = np.arange(vol * b * ncols)
    x = ((g % 7 - 3) + 1j * (g % 5 - 2)).astype(np.complex128)
    y0 = ((g % 3 - 1) + 1j * (g % 2)).astype(np.complex128)
    alpha, beta = 2.0 + 0j, -1.0 + 0j
    # reference: repeated oracle applications; y layout pxyztscn with p = power index
    refs, cur = [], x.copy()
    for _ in range(power):
        nxt = np.zeros_like(x)
        oracle_bsr(T_CDOUBLE, dim, 0, vol, b, b, ii, jj, vals, False, cur, ncols, True, nxt, ncols,
                   True, ncols, 1.0)
        refs.append(nxt)
        cur = nxt
    yref = np.concatenate([alpha * r + beta * y0 for r in refs])
    full = [([0] * 6, dim)]
    op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, spin, color], [1, 1, 1, 1, spin, color],
                       False, [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                       [torch.from_numpy(vals).to(gpu)])
    dimx = [1, L, L, L, L, spin, color, ncols]
    dimy = [power, L, L, L, L, spin, color, ncols]
    ty = torch.from_numpy(np.concatenate([y0] * power)).to(gpu)
    sb.bsr_krylov(alpha, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTSCn", [0] * 8, dimx,
                  dimx, [torch.from_numpy(x).to(gpu)], beta, [([0] * 8, dimy)], "pxyztscn",
                  [0] * 8, dimy, dimy, "p", [ty])
    torch.cuda.synchronize()
    op.destroy()
    assert rel_err(ty.cpu().numpy(), yref) < 1e-13


@pytest.mark.parametrize("spin,color,ncols,beta,power", [(1, 3, 2, 0.0, 1), (4, 3, 3, 0.5, 1),
                                                        (1, 3, 2, 1.0, 2)])
def test_bsr_image_side(gpu, spin, color, ncols, beta, power):
    """x with the image labels, y with the domain labels: y = alpha A^H x + beta y (the
    reference's transSp, bsr.h:1942, hipsparse CONJUGATE_TRANSPOSE)."""
    import torch
    import superbblas_amd as sb
    from _common import oracle_bsr_adjoint
    L = 4
    dim, ii, jj, vals, nb = lattice_operator(L, spin, color)
    b = spin * color
    vol = L ** 4
    n = vol * b * ncols
    g = np.arange(n)
    x = ((g % 7 - 3) + 1j * (g % 5 - 2)).astype(np.complex128)
    y0 = ((np.arange(n * power) % 3 - 1) + 1j).astype(np.complex128)
    alpha = 1 - 1j
    refs, cur = [], x
    for _ in range(power):
        nxt = np.zeros_like(x)
        oracle_bsr_adjoint(T_CDOUBLE, dim, 0, vol, b, b, ii, jj, vals, False, cur, ncols, True,
                           nxt, ncols, True, vol * b, ncols, 1.0)
        refs.append(nxt)
        cur = nxt
    yref = np.concatenate([alpha * r + beta * y0[p * n:(p + 1) * n] for p, r in enumerate(refs)])
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, spin, color]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, False, [torch.from_numpy(ii).to(gpu)],
                       [torch.from_numpy(jj).to(gpu)], [torch.from_numpy(vals).to(gpu)])
    dimx = [1, L, L, L, L, spin, color, ncols]
    dimy = [power] + dimx[1:]
    tx = torch.from_numpy(x).to(gpu)
    ty = torch.from_numpy(y0.copy()).to(gpu)
    sb.bsr_krylov(alpha, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pxyztscn", [0] * 8, dimx,
                  dimx, [tx], beta, [([0] * 8, dimy)], "pXYZTSCn", [0] * 8, dimy, dimy,
                  "p" if power > 1 else None, [ty])
    torch.cuda.synchronize()
    op.destroy()
    assert np.array_equal(ty.cpu().numpy(), yref)


@pytest.mark.parametrize("variant,pd", [(0, 1), (0, 2), (0, 3), (1, 1), (2, 1)])
@pytest.mark.parametrize("ncols,dtype", [(3, np.complex128), (16, np.complex64), (20, np.complex128),
                                         (5, np.float64), (12, np.complex64), (12, np.float32)])
def test_bsr_12x12_kernel_forms(gpu, variant, pd, ncols, dtype):
    """The 12x12 (spin x color) 9-point operator through every kernel form: the block-staged
    MFMA kernel (variant 0, row-major x with ncols <= 16; blocks staged by LDS-DMA 1-3 ahead,
    `bsr.blk_pd`, packed slots for 8-byte elements), the column-preloading MFMA kernel (variant
    2, and variant 0 beyond 16 columns) and the generic-row MFMA kernel (variant 1); exact."""
    import torch
    import superbblas_amd as sb
    from _common import TYPE_OF
    L, spin, color = 4, 4, 3
    dim, ii, jj, vals, nb = lattice_operator(L, spin, color, dtype)
    b = spin * color
    vol = L ** 4
    g = np.arange(vol * b * ncols)
    x = ((g % 9 - 4) + (1j * (g % 5 - 2) if np.dtype(dtype).kind == "c" else 0)).astype(dtype)
    yref = np.zeros(vol * b * ncols, dtype)
    oracle_bsr(TYPE_OF[np.dtype(dtype)], dim, 0, vol, b, b, ii, jj, vals, False, x, ncols, True,
               yref, ncols, True, ncols, 1.0)
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, spin, color]
    sb.tune_set("bsr.variant", variant)
    old_pd = sb.tune_get("bsr.blk_pd")
    sb.tune_set("bsr.blk_pd", pd)
    try:
        op = sb.create_bsr(full, dim, full, dim, blk, blk, False, [torch.from_numpy(ii).to(gpu)],
                           [torch.from_numpy(jj).to(gpu)], [torch.from_numpy(vals).to(gpu)])
        dimx = [1, L, L, L, L, spin, color, ncols]
        ty = torch.zeros(vol * b * ncols, dtype=getattr(torch, np.dtype(dtype).name), device=gpu)
        sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTSCn", [0] * 8, dimx,
                      dimx, [torch.from_numpy(x).to(gpu)], 0.0, [([0] * 8, dimx)], "pxyztscn",
                      [0] * 8, dimx, dimx, "p", [ty])
        torch.cuda.synchronize()
        op.destroy()
    finally:
        sb.tune_set("bsr.variant", 0)
        sb.tune_set("bsr.blk_pd", old_pd)
    assert np.array_equal(ty.cpu().numpy(), yref)


@pytest.mark.parametrize("pd", [1, 3])
@pytest.mark.parametrize("dtype,ncols,form", [(np.complex64, 16, 8), (np.complex64, 13, 8),
                                              (np.complex128, 12, 7)])
def test_bsr_12x12_skipped_blocks_dma(gpu, dtype, ncols, form, pd):
    """Blocks with column -1 on the LDS-DMA 12x12 kernel (packed slots for complex<float>): a
    skipped block's slot must not read past the caller's arrays -- with 13-16 rhs columns the x
    part of a packed complex<float> slot is longer than a value block, and the last block of the
    last row is skipped here -- and must contribute nothing (exact vs the oracle)."""
    import torch
    import superbblas_amd as sb
    from _common import TYPE_OF
    L, spin, color = 4, 4, 3
    dim, ii, jj, vals, nb = lattice_operator(L, spin, color, dtype)
    b = spin * color
    vol = L ** 4
    jj = jj.reshape(vol, nb, 6).copy()
    jj[::3, 1, :] = -1           # every third row skips its -x block
    jj[-1, nb - 1, :] = -1       # the very last block of the value array
    jj[-2, :, :] = -1            # a row with no blocks at all
    jj = jj.reshape(-1)
    g = np.arange(vol * b * ncols)
    x = ((g % 9 - 4) + 1j * (g % 5 - 2)).astype(dtype)
    yref = np.zeros(vol * b * ncols, dtype)
    oracle_bsr(TYPE_OF[np.dtype(dtype)], dim, 0, vol, b, b, ii, jj, vals, False, x, ncols, True,
               yref, ncols, True, ncols, 1.0)
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, spin, color]
    # the values exactly as long as the operator (no slack after the last block)
    tv = torch.from_numpy(vals).to(gpu)
    op = sb.create_bsr(full, dim, full, dim, blk, blk, False, [torch.from_numpy(ii).to(gpu)],
                       [torch.from_numpy(jj).to(gpu)], [tv])
    dimx = [1, L, L, L, L, spin, color, ncols]
    ty = torch.full((vol * b * ncols,), 3.0, dtype=getattr(torch, np.dtype(dtype).name), device=gpu)
    old_pd = sb.tune_get("bsr.blk_pd")
    sb.tune_set("bsr.blk_pd", pd)
    try:
        sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTSCn", [0] * 8, dimx,
                      dimx, [torch.from_numpy(x).to(gpu)], 0.0, [([0] * 8, dimx)], "pxyztscn",
                      [0] * 8, dimx, dimx, "p", [ty])
        torch.cuda.synchronize()
    finally:
        sb.tune_set("bsr.blk_pd", old_pd)
    used = sb.tune_get("bsr.last_kernel")
    op.destroy()
    assert used == form, used
    assert np.array_equal(ty.cpu().numpy(), yref)


@pytest.mark.parametrize("spin,color,ncols,form", [(1, 3, 12, 2), (1, 3, 2, 1), (4, 3, 3, 7),
                                                   (4, 3, 12, 7)])
def test_bsr_image_side_kernel_form(gpu, spin, color, ncols, form):
    """A^H products (x with the image labels) run the same specialised kernels as A (the
    transposed operator carries its domain extent), exact vs the oracle's adjoint loop."""
    import torch
    import superbblas_amd as sb
    from _common import oracle_bsr_adjoint
    L = 4
    dim, ii, jj, vals, nb = lattice_operator(L, spin, color)
    b = spin * color
    vol = L ** 4
    n = vol * b * ncols
    g = np.arange(n)
    x = ((g % 7 - 3) + 1j * (g % 5 - 2)).astype(np.complex128)
    yref = np.zeros(n, np.complex128)
    oracle_bsr_adjoint(T_CDOUBLE, dim, 0, vol, b, b, ii, jj, vals, False, x, ncols, True, yref,
                       ncols, True, vol * b, ncols, 1.0)
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, spin, color]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, False, [torch.from_numpy(ii).to(gpu)],
                       [torch.from_numpy(jj).to(gpu)], [torch.from_numpy(vals).to(gpu)])
    dimx = [1, L, L, L, L, spin, color, ncols]
    ty = torch.zeros(n, dtype=torch.complex128, device=gpu)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pxyztscn", [0] * 8, dimx, dimx,
                  [torch.from_numpy(x).to(gpu)], 0.0, [([0] * 8, dimx)], "pXYZTSCn", [0] * 8,
                  dimx, dimx, "p", [ty])
    torch.cuda.synchronize()
    used = sb.tune_get("bsr.last_kernel")
    op.destroy()
    assert used == form, used
    assert np.array_equal(ty.cpu().numpy(), yref)
