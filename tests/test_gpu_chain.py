"""The configs[4] propagator chain (bench.py chain_bench) checked stage by stage against the
oracle at a reduced lattice: (1) redistribute a complex<float> propagator `tnsxyzc` into the
operator's domain layout `pxyztscn` (copy, bit-exact), (2) apply the 9-point 12x12-block
(spin x color) BSR operator (bsr_krylov, bsr.h:2516-2543), (3) contract the result with its
conjugate over the lattice and color into `TSnsN` (contraction, dist.h:3701-3731).  Tolerances
are single precision (sums of <= 108 and <= 768 products).  The full-size run in bench.py
checks the Hermitian property of stage 3 instead."""
import numpy as np
import pytest

from _common import T_CFLOAT, oracle_bsr, oracle_contraction, oracle_copy, rel_err

pytestmark = pytest.mark.gpu


def _vol(d):
    n = 1
    for x in d:
        n *= x
    return n


def test_chain_reduced(gpu):
    import torch
    import superbblas_amd as sb
    rng = np.random.default_rng(11)
    Ls, Lt, ncols, s_, c_ = 4, 8, 3, 4, 3
    b = s_ * c_
    dims = [Ls, Ls, Ls, Lt]
    V = _vol(dims)
    cf = np.complex64

    def rand(n):
        return (rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)).astype(cf)

    # (1) tnsxyzc -> pxyztscn
    dsrc = [Lt, ncols, s_, Ls, Ls, Ls, c_]
    dx = [1, Ls, Ls, Ls, Lt, s_, c_, ncols]
    src = rand(_vol(dsrc))
    x_ref = np.zeros(_vol(dx), cf)
    oracle_copy(1.0, "tnsxyzc", [0] * 7, dsrc, dsrc, src, "pxyztscn", [0] * 8, dx, x_ref)
    t_src = torch.from_numpy(src).to(gpu)
    t_x = torch.zeros(_vol(dx), dtype=torch.complex64, device=gpu)
    sb.copy(1.0, [([0] * 7, dsrc)], "tnsxyzc", [0] * 7, dsrc, dsrc, [t_src], [([0] * 8, dx)],
            "pxyztscn", [0] * 8, dx, [t_x])
    torch.cuda.synchronize()
    assert np.array_equal(t_x.cpu().numpy().view(np.uint8), x_ref.view(np.uint8))

    # (2) y = A x, A the 9-point operator with 12x12 blocks
    sites = np.array(np.unravel_index(np.arange(V), dims)).T
    jj = np.zeros((V, 9, 6), np.int32)
    jj[:, 0, :4] = sites
    k = 1
    for d in range(4):
        for sg in (-1, 1):
            c = sites.copy()
            c[:, d] = (c[:, d] + sg) % dims[d]
            jj[:, k, :4] = c
            k += 1
    vals = rand(V * 9 * b * b)
    dim = dims + [s_, c_]
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, s_, c_]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, False,
                       [torch.full((V,), 9, dtype=torch.int32, device=gpu)],
                       [torch.from_numpy(jj.reshape(-1)).to(gpu)], [torch.from_numpy(vals).to(gpu)])
    t_y = torch.empty_like(t_x)
    p_x = [([0] * 8, dx)]
    sb.bsr_krylov(1.0, op, "XYZTSC", "xyztsc", p_x, "pxyztscn", [0] * 8, dx, dx, [t_x], 0.0, p_x,
                  "pXYZTSCn", [0] * 8, dx, dx, "p", [t_y])
    torch.cuda.synchronize()
    op.destroy()
    y_ref = np.zeros(_vol(dx), cf)
    oracle_bsr(T_CFLOAT, dim, 0, V, b, b, np.full(V, 9, np.int32), jj.reshape(-1), vals, False,
               x_ref, ncols, True, y_ref, ncols, True, ncols, 1.0)
    y = t_y.cpu().numpy()
    assert rel_err(y, y_ref) < 2e-6

    # (3) TSnsN = sum_{XYZC} conj(y[XYZT S C n]) y[XYZT s C N]
    dr = [Lt, s_, ncols, s_, ncols]
    t_r = torch.empty(_vol(dr), dtype=torch.complex64, device=gpu)
    sb.contraction(1.0, p_x, [0] * 8, dx, dx, "pXYZTSCn", True, [t_y], p_x, [0] * 8, dx, dx,
                   "pXYZTsCN", False, [t_y], 0.0, [([0] * 5, dr)], [0] * 5, dr, dr, "TSnsN", [t_r])
    torch.cuda.synchronize()
    r_ref = np.zeros(_vol(dr), cf)
    oracle_contraction(1.0, "pXYZTSCn", [0] * 8, dx, dx, True, y_ref, "pXYZTsCN", [0] * 8, dx, dx,
                       False, y_ref, 0.0, "TSnsN", [0] * 5, dr, dr, r_ref)
    r = t_r.cpu().numpy()
    assert rel_err(r, r_ref) < 2e-5
    h = r.reshape(Lt, s_ * ncols, s_ * ncols)
    assert rel_err(h, np.conj(np.transpose(h, (0, 2, 1)))) < 1e-5


def test_chain_full_size(gpu):
    """configs[4] at its full size (16^3 x 64 sites, n = 12, complex<float>; bench.py chain_bench)
    against a complex<double> reference computed with torch on the same GPU: the redistribution
    bit-exact, the 12x12-block 9-point operator within the rounding of its 108-term sums, and the
    TSnsN contraction (49 152-term sums) within single-precision accumulation."""
    import torch
    import superbblas_amd as sb
    Ls, Lt, ncols, s_, c_ = 16, 64, 12, 4, 3
    b = s_ * c_
    dims = [Ls, Ls, Ls, Lt]
    V = _vol(dims)
    g = torch.Generator(device=gpu).manual_seed(5)

    def rand(n):
        return torch.complex(torch.rand(n, generator=g, device=gpu) * 2 - 1,
                             torch.rand(n, generator=g, device=gpu) * 2 - 1)

    # (1) tnsxyzc -> pxyztscn
    dsrc = [Lt, ncols, s_, Ls, Ls, Ls, c_]
    dx = [1, Ls, Ls, Ls, Lt, s_, c_, ncols]
    src = rand(_vol(dsrc))
    t_x = torch.empty(_vol(dx), dtype=torch.complex64, device=gpu)
    sb.copy(1.0, [([0] * 7, dsrc)], "tnsxyzc", [0] * 7, dsrc, dsrc, [src], [([0] * 8, dx)],
            "pxyztscn", [0] * 8, dx, [t_x])
    torch.cuda.synchronize()
    x_ref = src.view(dsrc).permute(3, 4, 5, 0, 2, 6, 1).reshape(-1)
    assert torch.equal(t_x.view(torch.float32), x_ref.contiguous().view(torch.float32))
    del src, x_ref

    # (2) y = A x, the 9-point operator with 12x12 blocks
    sites = np.array(np.unravel_index(np.arange(V), dims)).T
    jj = np.zeros((V, 9, 6), np.int32)
    nb = np.zeros((V, 9), np.int64)
    jj[:, 0, :4] = sites
    nb[:, 0] = np.arange(V)
    k = 1
    for d in range(4):
        for sg in (-1, 1):
            c = sites.copy()
            c[:, d] = (c[:, d] + sg) % dims[d]
            jj[:, k, :4] = c
            nb[:, k] = np.ravel_multi_index(c.T, dims)
            k += 1
    vals = rand(V * 9 * b * b)
    dim = dims + [s_, c_]
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, s_, c_]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, False,
                       [torch.full((V,), 9, dtype=torch.int32, device=gpu)],
                       [torch.from_numpy(jj.reshape(-1)).to(gpu)], [vals])
    t_y = torch.empty_like(t_x)
    p_x = [([0] * 8, dx)]
    sb.bsr_krylov(1.0, op, "XYZTSC", "xyztsc", p_x, "pxyztscn", [0] * 8, dx, dx, [t_x], 0.0, p_x,
                  "pXYZTSCn", [0] * 8, dx, dx, "p", [t_y])
    torch.cuda.synchronize()
    op.destroy()
    A = vals.view(V, 9, b, b)
    X = t_x.view(V, b, ncols)
    nbt = torch.from_numpy(nb).to(gpu)
    y_ref = torch.empty(V, b, ncols, dtype=torch.complex128, device=gpu)
    for c0 in range(0, V, 16384):  # (chunks: the gathered neighbours in complex<double>)
        c1 = min(V, c0 + 16384)
        y_ref[c0:c1] = torch.einsum("vkij,vkjn->vin", A[c0:c1].to(torch.complex128),
                                    X[nbt[c0:c1]].to(torch.complex128))
    err = (torch.linalg.vector_norm(t_y.view(V, b, ncols).to(torch.complex128) - y_ref) /
           torch.linalg.vector_norm(y_ref)).item()
    assert err < 1e-6, err
    del A, vals, X

    # (3) TSnsN = sum_{XYZC} conj(y[XYZT S C n]) y[XYZT s C N]
    dr = [Lt, s_, ncols, s_, ncols]
    t_r = torch.empty(_vol(dr), dtype=torch.complex64, device=gpu)
    sb.contraction(1.0, p_x, [0] * 8, dx, dx, "pXYZTSCn", True, [t_y], p_x, [0] * 8, dx, dx,
                   "pXYZTsCN", False, [t_y], 0.0, [([0] * 5, dr)], [0] * 5, dr, dr, "TSnsN", [t_r])
    torch.cuda.synchronize()
    yv = y_ref.view(Ls * Ls * Ls, Lt, s_, c_, ncols)
    r_ref = torch.einsum("XTSCn,XTsCN->TSnsN", yv.conj(), yv).reshape(-1)
    err = (torch.linalg.vector_norm(t_r.to(torch.complex128) - r_ref) /
           torch.linalg.vector_norm(r_ref)).item()
    assert err < 1e-5, err
