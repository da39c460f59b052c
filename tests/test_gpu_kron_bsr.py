"""Kronecker BSR (create_kron_bsr, bsr.h:2476-2490; builtin operator bsr.h:587-648) on the GPU vs
the oracle's restatement, on the 9-point lattice stencil with color blocks and one spin matrix
per direction (tests/bsr.cpp:547-644).  Integer-valued data: exact in every type."""
import numpy as np
import pytest

from _common import T_CDOUBLE, oracle_kron_bsr

pytestmark = pytest.mark.gpu


def kron_lattice(L, spin, color, sparse_kron=False):
    V = L ** 4
    sites = np.array(np.unravel_index(np.arange(V), (L, L, L, L))).T
    jj = []
    for s in sites:
        jj.append(list(s) + [0, 0])
        for d in range(4):
            for dr in (-1, 1):
                c = s.copy()
                c[d] = (c[d] + dr) % L
                jj.append(list(c) + [0, 0])
    jj = np.array(jj, np.int32).ravel()
    k = np.arange(V * 9 * color * color, dtype=np.int64)
    vals = ((k * 3 + 1) % 7 - 3) + 1j * ((k * 5 + 2) % 9 - 4)
    q = np.arange(9 * spin * spin, dtype=np.int64)
    kron = ((q * 5 + 2) % 7 - 3) + 1j * ((q * 3 + 1) % 5 - 2)
    if sparse_kron:
        # Wilson-projector-like pattern: half of every spin matrix is zero (the skip path)
        a, b = np.unravel_index(q % (spin * spin), (spin, spin))
        kron[(a + b + q // (spin * spin)) % 2 == 1] = 0
    return np.full(V, 9, np.int32), jj, vals, kron


def reference(L, spin, color, ncols, vals, kron, jj, x, alpha, beta, y0, power, bif=False):
    V = L ** 4
    cur, out = x.astype(np.complex128), []
    for p in range(power):
        y = np.zeros_like(cur)
        oracle_kron_bsr(T_CDOUBLE, [L, L, L, L, 1, 1], 0, V, 9, color, color, spin, spin, jj,
                        vals, kron, bif, cur, y, ncols, 1.0)
        out.append(y)
        cur = y
    return np.concatenate([alpha * o + beta * y0[i * len(x):(i + 1) * len(x)]
                           for i, o in enumerate(out)])


@pytest.mark.parametrize("dtype", [np.complex128, np.complex64, np.float64, np.float32])
@pytest.mark.parametrize("spin,color,ncols", [(4, 3, 3), (2, 3, 2), (4, 1, 5)])
def test_kron_types_sizes(gpu, dtype, spin, color, ncols):
    """(4, 3) runs the specialized kernel, the others the generic one."""
    import torch
    import superbblas_amd as sb
    L = 4
    cplx = np.dtype(dtype).kind == "c"
    ii, jj, vals, kron = kron_lattice(L, spin, color)
    if not cplx:
        vals, kron = vals.real.copy(), kron.real.copy()
    V = L ** 4
    g = np.arange(V * color * ncols * spin)
    x = ((g % 7 - 3) + (1j * (g % 5 - 2) if cplx else 0)).astype(np.complex128)
    ref = reference(L, spin, color, ncols, vals.astype(np.complex128),
                    kron.astype(np.complex128), jj, x, 1.0, 0.0, np.zeros_like(x), 1)
    dim = [L, L, L, L, spin, color]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, False,
                            [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                            [torch.from_numpy(vals.astype(dtype)).to(gpu)],
                            [torch.from_numpy(kron.astype(dtype)).to(gpu)])
    dimx = [1, L, L, L, L, color, ncols, spin]
    tx = torch.from_numpy((x if cplx else x.real).astype(dtype)).to(gpu)
    ty = torch.zeros(V * color * ncols * spin, dtype=tx.dtype, device=gpu)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTCnS", [0] * 8, dimx,
                  dimx, [tx], 0.0, [([0] * 8, dimx)], "pxyztcns", [0] * 8, dimx, dimx, "p", [ty])
    torch.cuda.synchronize()
    op.destroy()
    out = ty.cpu().numpy().astype(np.complex128)
    assert np.array_equal(out, ref if cplx else ref.real.astype(np.complex128))


@pytest.mark.parametrize("bif", [False, True])
def test_kron_sparse_alpha_beta_power(gpu, bif):
    """Sparse spin matrices, complex alpha, beta != 0, powers, both block orders."""
    import torch
    import superbblas_amd as sb
    L, spin, color, ncols, power = 4, 4, 3, 2, 3
    ii, jj, vals, kron = kron_lattice(L, spin, color, sparse_kron=True)
    V = L ** 4
    n = V * color * ncols * spin
    g = np.arange(n)
    x = ((g % 5 - 2) + 1j * (g % 3 - 1)).astype(np.complex128)
    y0 = ((np.arange(n * power) % 7 - 3) + 1j).astype(np.complex128)
    alpha, beta = 1 - 1j, 2.0
    ref = reference(L, spin, color, ncols, vals, kron, jj, x, alpha, beta, y0, power, bif)
    dim = [L, L, L, L, spin, color]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, bif,
                            [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                            [torch.from_numpy(vals).to(gpu)], [torch.from_numpy(kron).to(gpu)])
    dimx = [1, L, L, L, L, color, ncols, spin]
    dimy = [power] + dimx[1:]
    tx = torch.from_numpy(x).to(gpu)
    ty = torch.from_numpy(y0.copy()).to(gpu)
    sb.bsr_krylov(alpha, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTCnS", [0] * 8, dimx,
                  dimx, [tx], beta, [([0] * 8, dimy)], "pxyztcns", [0] * 8, dimy, dimy, "p", [ty])
    torch.cuda.synchronize()
    op.destroy()
    assert np.array_equal(ty.cpu().numpy(), ref)


def test_kron_other_layouts(gpu):
    """x and y in layouts other than the preferred (D, d, C, kd): through the temporaries."""
    import torch
    import superbblas_amd as sb
    L, spin, color, ncols = 4, 4, 3, 3
    ii, jj, vals, kron = kron_lattice(L, spin, color)
    V = L ** 4
    g = np.arange(V * color * ncols * spin)
    x = ((g % 7 - 3) + 1j * (g % 5 - 2)).astype(np.complex128)
    ref = reference(L, spin, color, ncols, vals, kron, jj, x, 1.0, 0.0, np.zeros_like(x), 1)
    # preferred layouts: x pXYZTCnS and y pxyztcns; use x = nXYZTSC (column major) and
    # y = pxyztsnc instead
    xt = x.reshape(L, L, L, L, color, ncols, spin).transpose(5, 0, 1, 2, 3, 6, 4).copy()
    dim = [L, L, L, L, spin, color]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, False,
                            [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                            [torch.from_numpy(vals).to(gpu)], [torch.from_numpy(kron).to(gpu)])
    dimx = [ncols, L, L, L, L, spin, color]
    dimy = [1, L, L, L, L, spin, ncols, color]
    tx = torch.from_numpy(xt.ravel()).to(gpu)
    ty = torch.zeros(V * color * ncols * spin, dtype=torch.complex128, device=gpu)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 7, dimx)], "nXYZTSC", [0] * 7, dimx,
                  dimx, [tx], 0.0, [([0] * 8, dimy)], "pxyztsnc", [0] * 8, dimy, dimy, "p", [ty])
    torch.cuda.synchronize()
    op.destroy()
    out = ty.cpu().numpy().reshape(L, L, L, L, spin, ncols, color).transpose(0, 1, 2, 3, 6, 5, 4)
    assert np.array_equal(out.ravel(), ref)


def test_kron_errors(gpu):
    import torch
    import superbblas_amd as sb
    L, spin, color = 4, 4, 3
    ii, jj, vals, kron = kron_lattice(L, spin, color)
    dim = [L, L, L, L, spin, color]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    t = lambda a: torch.from_numpy(a).to(gpu)  # noqa: E731
    ii2 = ii.copy()
    ii2[0], ii2[1] = 8, 10
    with pytest.raises(sb.SuperbblasError, match="different number of nonzeros"):
        sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, False, [t(ii2)], [t(jj)],
                           [t(vals)], [t(kron)])
    jj2 = jj.copy()
    jj2[6] = -1
    with pytest.raises(sb.SuperbblasError, match="-1"):
        sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, False, [t(ii)], [t(jj2)],
                           [t(vals)], [t(kron)])
    with pytest.raises(sb.SuperbblasError, match="simultaneous blocking"):
        sb.create_kron_bsr(full, dim, full, dim, blk, blk, [1, 1, 1, 1, spin, color],
                           [1, 1, 1, 1, spin, color], False, [t(ii)], [t(jj)], [t(vals)],
                           [t(kron)])


@pytest.mark.parametrize("ncols,L", [(8, 4), (12, 4), (12, 3), (16, 4), (17, 4), (40, 4)])
@pytest.mark.parametrize("bif,sparse", [(False, False), (True, True)])
def test_kron_mfma_kernel(gpu, ncols, L, bif, sparse):
    """complex<double> 3x3 x 4x4 from 8 rhs columns: the spin products on the matrix cores
    (bsr_kron_mfma_kernel; 16-column groups, partial last group; bsr_kron_mfma_packed_kernel at 8
    and 12 columns: a wave's 16 column slots over several rows; x staged by LDS-DMA 1-3
    neighbours ahead or loaded per lane, y written per lane or through the same ring; 3^4 sites: a last workgroup with
    fewer rows than its slots), complex alpha, beta,
    powers; integer data, exact; and the same results with each form switched off."""
    import torch
    import superbblas_amd as sb
    spin, color, power = 4, 3, 2
    ii, jj, vals, kron = kron_lattice(L, spin, color, sparse_kron=sparse)
    V = L ** 4
    n = V * color * ncols * spin
    g = np.arange(n)
    x = ((g % 5 - 2) + 1j * (g % 3 - 1)).astype(np.complex128)
    y0 = ((np.arange(n * power) % 7 - 3) + 1j).astype(np.complex128)
    alpha, beta = 1 - 1j, 2.0
    ref = reference(L, spin, color, ncols, vals, kron, jj, x, alpha, beta, y0, power, bif)
    dim = [L, L, L, L, spin, color]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, bif,
                            [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                            [torch.from_numpy(vals).to(gpu)], [torch.from_numpy(kron).to(gpu)])
    dimx = [1, L, L, L, L, color, ncols, spin]
    dimy = [power] + dimx[1:]
    outs = []
    old_xl, old_yl = sb.tune_get("bsr.kron_xlds"), sb.tune_get("bsr.kron_ylds")
    old_spin = sb.tune_get("bsr.kron_spin")
    sb.tune_set("bsr.kron_spin", 0)  # the MFMA forms (the opt-in spin-first kernel: test_kron_spin_kernel)
    try:
        # packed column slots (8 and 12 columns: several rows per wave), one row per wave, no MFMA
        # (MFMA kernels, packed slots, x staging depth, y staged)
        for on, pack, xl, yl in ((1, 1, 1, 0), (1, 1, 2, 1), (1, 1, 3, 0), (1, 1, 0, 0),
                                 (1, 0, 2, 1), (1, 0, 3, 0), (1, 0, 0, 0), (0, 1, 1, 1)):
            sb.tune_set("bsr.kron_mfma", on)
            sb.tune_set("bsr.kron_pack", pack)
            sb.tune_set("bsr.kron_xlds", xl)
            sb.tune_set("bsr.kron_ylds", yl)
            ty = torch.from_numpy(y0.copy()).to(gpu)
            sb.bsr_krylov(alpha, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTCnS", [0] * 8,
                          dimx, dimx, [torch.from_numpy(x).to(gpu)], beta, [([0] * 8, dimy)],
                          "pxyztcns", [0] * 8, dimy, dimy, "p", [ty])
            torch.cuda.synchronize()
            outs.append((sb.tune_get("bsr.last_kernel"), ty.cpu().numpy()))
    finally:
        sb.tune_set("bsr.kron_mfma", 1)
        sb.tune_set("bsr.kron_pack", 1)
        sb.tune_set("bsr.kron_xlds", old_xl)
        sb.tune_set("bsr.kron_ylds", old_yl)
        sb.tune_set("bsr.kron_spin", old_spin)
        op.destroy()
    packed = 6 if ncols in (8, 12) else 5
    assert [o[0] for o in outs[:7]] == [packed] * 4 + [5] * 3 and outs[7][0] not in (5, 6)
    for form, out in outs:
        assert np.array_equal(out, ref), form


@pytest.mark.parametrize("seed", range(24))
def test_kron_fuzz(gpu, seed):
    """Random Kronecker operators: lattice 1-4, spin 1 / 2 / 4, color 1-3, rhs columns 1-300
    (log-uniform), every type, either block order, sparse or dense spin matrices; so every Kron
    kernel form (MFMA, packed MFMA, LDS, generic) meets ragged column counts.  Exact."""
    import torch
    import superbblas_amd as sb
    rng = np.random.default_rng(3100 + seed)
    dtype = [np.complex128, np.complex64, np.float64, np.float32][seed % 4]
    cplx = np.dtype(dtype).kind == "c"
    L = int(rng.integers(1, 5))
    spin = int(rng.choice([1, 2, 4]))
    color = int(rng.choice([1, 2, 3, 3]))
    if seed % 3 == 0:
        spin, color = 4, 3  # the specialised kernels
    ncols = int(np.exp(rng.uniform(0, np.log(300))))
    bif = bool(rng.integers(0, 2))
    ii, jj, vals, kron = kron_lattice(L, spin, color, sparse_kron=bool(rng.integers(0, 2)))
    if not cplx:
        vals, kron = vals.real.copy(), kron.real.copy()
    V = L ** 4
    g = np.arange(V * color * ncols * spin)
    x = ((g % 7 - 3) + (1j * (g % 5 - 2) if cplx else 0)).astype(np.complex128)
    ref = reference(L, spin, color, ncols, vals.astype(np.complex128),
                    kron.astype(np.complex128), jj, x, 1.0, 0.0, np.zeros_like(x), 1, bif=bif)
    dim = [L, L, L, L, spin, color]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, bif,
                            [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                            [torch.from_numpy(vals.astype(dtype)).to(gpu)],
                            [torch.from_numpy(kron.astype(dtype)).to(gpu)])
    dimx = [1, L, L, L, L, color, ncols, spin]
    tx = torch.from_numpy((x if cplx else x.real).astype(dtype)).to(gpu)
    ty = torch.zeros(V * color * ncols * spin, dtype=tx.dtype, device=gpu)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTCnS", [0] * 8, dimx,
                  dimx, [tx], 0.0, [([0] * 8, dimx)], "pxyztcns", [0] * 8, dimx, dimx, "p", [ty])
    torch.cuda.synchronize()
    kind = sb.tune_get("bsr.last_kernel")
    op.destroy()
    out = ty.cpu().numpy().astype(np.complex128)
    assert np.array_equal(out, ref if cplx else ref.real.astype(np.complex128)), \
        (dtype, L, spin, color, ncols, bif, kind)


def wilson_spin():
    """1, 1 -+ gamma_mu (chiral basis): the bench's spin matrices (bench.py wilson_bench)"""
    i_ = 1j
    g = [np.array([[0, 0, 0, i_], [0, 0, i_, 0], [0, -i_, 0, 0], [-i_, 0, 0, 0]]),
         np.array([[0, 0, 0, -1], [0, 0, 1, 0], [0, 1, 0, 0], [-1, 0, 0, 0]]),
         np.array([[0, 0, i_, 0], [0, 0, 0, -i_], [-i_, 0, 0, 0], [0, i_, 0, 0]]),
         np.array([[0, 0, 1, 0], [0, 0, 0, 1], [1, 0, 0, 0], [0, 1, 0, 0]])]
    ks = [np.eye(4)]
    for gm in g:
        ks += [np.eye(4) - gm, np.eye(4) + gm]
    return np.array(ks, np.complex128).ravel()


@pytest.mark.parametrize("ncols,L", [(8, 4), (12, 4), (12, 3), (13, 3), (16, 5), (40, 2), (64, 4)])
@pytest.mark.parametrize("bif,kind", [(False, "dense"), (True, "sparse"), (False, "wilson"),
                                      (True, "wilson"), (False, "thin")])
def test_kron_spin_kernel(gpu, ncols, L, bif, kind):
    """complex<double> 3x3 x 4x4 from 8 rhs columns, spin first on the VALU (bsr_kron_spin_kernel:
    a lane per (row, column) pair, so pairs run across row boundaries and the last wave is
    ragged at every column count; every spin row as two terms from the operator's table; rows
    in the XCD order or not) when no spin row has more than two nonzeros (sparse: two per row;
    Wilson projectors; thin: rows with one nonzero and zero rows), the MFMA kernels otherwise
    (dense); complex alpha, beta, powers; integer data: exact, the same bits with the XCD order
    off and the same values as the MFMA kernels."""
    import torch
    import superbblas_amd as sb
    spin, color, power = 4, 3, 2
    ii, jj, vals, kron = kron_lattice(L, spin, color, sparse_kron=kind == "sparse")
    if kind == "wilson":
        kron = wilson_spin()
    if kind == "thin":
        kron = kron.reshape(9, 4, 4).copy()
        kron[:, :, 1:] = 0           # one nonzero per row
        kron[::2, 2, :] = 0          # and zero rows
        kron = kron.ravel()
    if bif and kind == "wilson":
        kron = kron.reshape(9, 4, 4).transpose(0, 2, 1).ravel().copy()
    V = L ** 4
    n = V * color * ncols * spin
    g = np.arange(n)
    x = ((g % 5 - 2) + 1j * (g % 3 - 1)).astype(np.complex128)
    y0 = ((np.arange(n * power) % 7 - 3) + 1j).astype(np.complex128)
    alpha, beta = 1 - 1j, 2.0
    ref = reference(L, spin, color, ncols, vals, kron, jj, x, alpha, beta, y0, power, bif)
    dim = [L, L, L, L, spin, color]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, bif,
                            [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                            [torch.from_numpy(vals).to(gpu)], [torch.from_numpy(kron).to(gpu)])
    dimx = [1, L, L, L, L, color, ncols, spin]
    dimy = [power] + dimx[1:]
    outs = []
    try:
        for spin_on, order in ((1, 1), (1, 0), (0, 1), (2, 1), (2, 0)):
            sb.tune_set("bsr.kron_spin", spin_on)
            sb.tune_set("bsr.kron_order", order)
            ty = torch.from_numpy(y0.copy()).to(gpu)
            sb.bsr_krylov(alpha, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTCnS", [0] * 8,
                          dimx, dimx, [torch.from_numpy(x).to(gpu)], beta, [([0] * 8, dimy)],
                          "pxyztcns", [0] * 8, dimy, dimy, "p", [ty])
            torch.cuda.synchronize()
            outs.append((sb.tune_get("bsr.last_kernel"), ty.cpu().numpy()))
    finally:
        sb.tune_set("bsr.kron_spin", 0)
        sb.tune_set("bsr.kron_order", 1)
        op.destroy()
    spin_form = 9 if kind != "dense" else outs[2][0]
    xor_form = 12 if kind == "wilson" else outs[2][0]  # (diagonal + XOR partner: Wilson only)
    assert outs[0][0] == spin_form and outs[1][0] == spin_form and outs[2][0] not in (9, 12)
    assert outs[3][0] == xor_form and outs[4][0] == xor_form
    for form, out in outs:
        assert np.array_equal(out, ref), form


def test_kron_spin_random_values(gpu):
    """random values (16^4 would be the bench; 6^4 here): the spin-first kernel within rounding
    of the oracle and of the color-first MFMA kernel (the sums are associated differently)"""
    import torch
    import superbblas_amd as sb
    L, spin, color, ncols = 6, 4, 3, 12
    rng = np.random.default_rng(11)
    ii, jj, _, _ = kron_lattice(L, spin, color)
    V = L ** 4
    vals = rng.standard_normal(V * 81) + 1j * rng.standard_normal(V * 81)
    kron = wilson_spin()
    x = rng.standard_normal(V * 12 * ncols) + 1j * rng.standard_normal(V * 12 * ncols)
    ref = reference(L, spin, color, ncols, vals, kron, jj, x, 1.0, 0.0, np.zeros_like(x), 1)
    dim = [L, L, L, L, spin, color]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, False,
                            [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                            [torch.from_numpy(vals).to(gpu)], [torch.from_numpy(kron).to(gpu)])
    dimx = [1, L, L, L, L, color, ncols, spin]
    outs = []
    try:
        for on in (1, 0, 2):
            sb.tune_set("bsr.kron_spin", on)
            ty = torch.zeros(V * 12 * ncols, dtype=torch.complex128, device=gpu)
            sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTCnS", [0] * 8,
                          dimx, dimx, [torch.from_numpy(x).to(gpu)], 0.0, [([0] * 8, dimx)],
                          "pxyztcns", [0] * 8, dimx, dimx, "p", [ty])
            torch.cuda.synchronize()
            outs.append(ty.cpu().numpy())
    finally:
        sb.tune_set("bsr.kron_spin", 0)
        op.destroy()
    scale = np.abs(ref).max()
    for out in outs:
        assert np.abs(out - ref).max() / scale < 1e-14


def dirac_pauli_spin():
    """1, 1 -+ gamma_mu in the Dirac-Pauli basis: gamma_4 diagonal, gamma_k = [[0, s_k], [-s_k, 0]]
    (rows nonzero at a and a ^ 3 or a ^ 2, or only at a)"""
    s1 = np.array([[0, 1], [1, 0]])
    s2 = np.array([[0, -1j], [1j, 0]])
    s3 = np.array([[1, 0], [0, -1]])
    z = np.zeros((2, 2))
    g = [np.block([[z, sk], [-sk, z]]) for sk in (s1, s2, s3)]
    g.append(np.diag([1, 1, -1, -1]))
    ks = [np.eye(4)]
    for gm in g:
        ks += [np.eye(4) - gm, np.eye(4) + gm]
    return np.array(ks, np.complex128).ravel()


@pytest.mark.parametrize("ncols", [8, 12, 20])
def test_kron_xor_kernel_dirac_pauli(gpu, ncols):
    """the diagonal + XOR-partner kernel (bsr.kron_spin 2) takes the Dirac-Pauli projectors too
    (a diagonal one among them: no partner); integer data, exact against the oracle"""
    import torch
    import superbblas_amd as sb
    L, spin, color = 4, 4, 3
    ii, jj, vals, _ = kron_lattice(L, spin, color)
    kron = dirac_pauli_spin()
    V = L ** 4
    g = np.arange(V * color * ncols * spin)
    x = ((g % 5 - 2) + 1j * (g % 3 - 1)).astype(np.complex128)
    ref = reference(L, spin, color, ncols, vals, kron, jj, x, 1.0, 0.0, np.zeros_like(x), 1)
    dim = [L, L, L, L, spin, color]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, False,
                            [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj).to(gpu)],
                            [torch.from_numpy(vals).to(gpu)], [torch.from_numpy(kron).to(gpu)])
    dimx = [1, L, L, L, L, color, ncols, spin]
    ty = torch.zeros(V * 12 * ncols, dtype=torch.complex128, device=gpu)
    try:
        sb.tune_set("bsr.kron_spin", 2)
        sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTCnS", [0] * 8, dimx,
                      dimx, [torch.from_numpy(x).to(gpu)], 0.0, [([0] * 8, dimx)], "pxyztcns",
                      [0] * 8, dimx, dimx, "p", [ty])
        torch.cuda.synchronize()
        used = sb.tune_get("bsr.last_kernel")
    finally:
        sb.tune_set("bsr.kron_spin", 0)
        op.destroy()
    assert used == 12
    assert np.array_equal(ty.cpu().numpy(), ref)
