"""One rank of the multi-process GPU parity run (launched by tests/test_gpu_dist.py through
torch.distributed.run).  Every rank holds its components on the GPU; the library redistributes
them through its communicator (RCCL, or the host-staged transport so several ranks can share one
GPU); rank 0 gathers the results and compares them with the oracle on the global tensors.

Cases (all multi-rank: the exchange, pack/unpack kernels and reductions run for real):
  copy   -- lattice field distributed over t, copied permuted/shifted/wrapped into a tensor
            distributed over x (Copy and Add)  [dist.h:2264-2438]
  contr  -- tnsxyzc x tNSxyzc -> tNSns with v0 split over z, v1 split over t (redistributed),
            output on rank 0 (cross-rank reduction) and output split over t with beta != 0
            [dist.h:3092-3196]
  bsr    -- 9-point stencil operator split over t with a halo domain partition, x split over t,
            y split over t, one power and two  [bsr.h:2107-2266]
  kron   -- the same stencil as a Kronecker operator (color blocks x spin matrices), two powers
            [bsr.h:2476-2490, 587-648]
  dense  -- cholesky / gesm with the matrices split over ranks  [dense.h:1007-1157]
  storage -- every rank saves its part of a tensor into one shared S3T file (global and block
            checksums), the file is checked by the S3T restatement, then loaded back into
            another distribution  [storage.h:1198-1385, 2142-2370]
  golden -- the reference's random-valued golden contractions (configs[0] 8^4 n=16, near-real,
            41-binade range; tests/golden cases 51-55) with the lattice split over the ranks as
            the bench's configs[3] shapes: v0 and v1 on an xyz grid (2x1x1, 2x2x1, ...; "4a") or
            v1 over t only ("4b", redistributed), output on rank 0; within 1e-10 per component
  split  -- the reference's split operator: a halo piece applied with a deferred request (its
            exchange in flight) and a core piece with just_local, then wait; a deferred copy
            [tests/bsr.cpp:402-545, 779-818; bsr.h:2199-2257, 2352-2359; dist.h:54-61]
  peer   -- two components per rank (the reference's --components=2, tests/contract.cpp:452-461)
            through the several-GPUs-per-rank path (pack on the origin device, hipMemcpyPeerAsync,
            unpack on the destination device; dist.h:205-241) forced on the one device of a test
            box by the tune key dist.force_peer: copies between t- and x-split tensors and the
            golden contractions, bit-exact / within 1e-10
  fuzz   -- seeded random copies (permutation, wrapping box, Copy/Add, type pairs) and
            contractions (label groups, orders, boxes, conj, alpha/beta) between random
            distributions over the ranks (some ranks may own nothing)
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from _common import (T_CDOUBLE, oracle_bsr, oracle_contraction, oracle_copy,  # noqa: E402
                     oracle_kron_bsr, rel_err)
from _golden import (component_errors, contraction_inputs, gen, manifest, output,  # noqa: E402
                     piece, put_piece, vol)


def scatter(sb, glob, dim, p, rank, nc, dev):
    return [torch.from_numpy(piece(glob, dim, *p[rank * nc + i])).to(dev) for i in range(nc)]


def gather(glob_init, dim, p, nc, local):
    """Every rank contributes its components; returns the assembled global tensor on all ranks."""
    mine = [t.cpu().numpy() for t in local]
    allc = [None] * dist.get_world_size()
    dist.all_gather_object(allc, mine)
    g = glob_init.copy()
    for rk, comps in enumerate(allc):
        for i, c in enumerate(comps):
            f, s = p[rk * nc + i]
            if vol(s):
                put_piece(g, dim, f, s, c)
    return g


def case_copy(sb, comm, rank, n, dev):
    dim0, dim1 = [4, 4, 2, 6], [6, 2, 4, 4]
    p0 = sb.basic_partitioning("xyzt", dim0, [1, 1, 1, n], "t", n, 1)
    p1 = sb.basic_partitioning("tzyx", dim1, [1, 1, 1, n], "x", n, 1)
    g0 = gen("index", vol(dim0), 1, np.complex128)
    for add in (False, True):
        g1 = gen("int", vol(dim1), 2, np.complex128)
        v0 = scatter(sb, g0, dim0, p0, rank, 1, dev)
        v1 = scatter(sb, g1, dim1, p1, rank, 1, dev)
        sb.copy(2.0 if add else 1.0, p0, "xyzt", [1, 2, 0, 3], [3, 4, 2, 5], dim0, v0, p1,
                "tzyx", [2, 0, 1, 3], dim1, v1, copyadd=sb.Add if add else sb.Copy, comm=comm)
        torch.cuda.synchronize()
        out = gather(np.zeros_like(g1), dim1, p1, 1, v1)
        ref = g1.copy()
        oracle_copy(2.0 if add else 1.0, "xyzt", [1, 2, 0, 3], [3, 4, 2, 5], dim0, g0, "tzyx",
                    [2, 0, 1, 3], dim1, ref, add=add)
        # untouched destination elements live in their owner's component: compare everything
        assert np.array_equal(out.view(np.uint8), ref.view(np.uint8)), ("copy", add)
    # masked (parity masks selecting the same elements on both sides, dist.h:3534-3602)
    from _golden import parity_masks
    case = {"o0": "xyzt", "o1": "tzyx", "dim0": dim0, "dim1": dim1, "from0": [1, 2, 0, 3],
            "from1": [2, 0, 1, 3]}
    gm0, gm1 = parity_masks(case)
    for add in (False, True):
        g1 = gen("int", vol(dim1), 2, np.complex128)
        v0 = scatter(sb, g0, dim0, p0, rank, 1, dev)
        v1 = scatter(sb, g1, dim1, p1, rank, 1, dev)
        m0 = scatter(sb, gm0, dim0, p0, rank, 1, dev)
        m1 = scatter(sb, gm1, dim1, p1, rank, 1, dev)
        sb.copy(1.0, p0, "xyzt", [1, 2, 0, 3], [3, 4, 2, 5], dim0, v0, p1, "tzyx", [2, 0, 1, 3],
                dim1, v1, copyadd=sb.Add if add else sb.Copy, comm=comm, mask0=m0, mask1=m1)
        torch.cuda.synchronize()
        out = gather(np.zeros_like(g1), dim1, p1, 1, v1)
        ref = g1.copy()
        oracle_copy(1.0, "xyzt", [1, 2, 0, 3], [3, 4, 2, 5], dim0, g0, "tzyx", [2, 0, 1, 3],
                    dim1, ref, add=add, mask0=gm0, mask1=gm1)
        assert np.array_equal(out.view(np.uint8), ref.view(np.uint8)), ("masked copy", add)


def case_contraction(sb, comm, rank, n, dev):
    L, nn = 4, 2
    d0 = [L, nn, 4, L, L, L * n, 3]  # tnsxyzc, z grows with the ranks (weak scaling)
    dr = [L, nn, 4, nn, 4]  # tNSns
    p0 = sb.basic_partitioning("tnsxyzc", d0, [1, 1, 1, 1, 1, n, 1], "z", n, 1)
    p1 = sb.basic_partitioning("tNSxyzc", d0, [n, 1, 1, 1, 1, 1, 1], "t", n, 1)
    g0 = gen("int", vol(d0), 1, np.complex128)
    g1 = gen("int", vol(d0), 2, np.complex128)
    v0 = scatter(sb, g0, d0, p0, rank, 1, dev)
    v1 = scatter(sb, g1, d0, p1, rank, 1, dev)
    z7, z5 = [0] * 7, [0] * 5
    # (a) output on rank 0 only, beta = 0
    pr = [([0] * 5, dr)] + [([0] * 5, [0] * 5)] * (n - 1)
    gr = gen("int", vol(dr), 3, np.complex128)
    vr = scatter(sb, gr, dr, pr, rank, 1, dev)
    if vr[0].numel() == 0:
        vr = [torch.zeros(1, dtype=torch.complex128, device=dev)]
    sb.timings_enable(True)
    sb.timings_reset()
    sb.contraction(1.0, p0, z7, d0, d0, "tnsxyzc", False, v0, p1, z7, d0, d0, "tNSxyzc", False,
                   v1, 0.0, pr, z5, dr, dr, "tNSns", vr, comm=comm)
    torch.cuda.synchronize()
    # the cross-rank reduction is pipelined: one GEMM per chunk of t (4 chunks of 1)
    assert sb.timings_get("gemm")[1] == L, sb.timings_report()
    sb.timings_enable(False)
    out = gather(np.zeros_like(gr), dr, pr, 1, vr[:1] if rank == 0 else [vr[0][:0]])
    ref = np.zeros_like(gr)
    oracle_contraction(1.0, "tnsxyzc", z7, d0, d0, False, g0, "tNSxyzc", z7, d0, d0, False, g1,
                       0.0, "tNSns", z5, dr, dr, ref)
    assert np.array_equal(out, ref), "contraction (a)"
    # (b) output split over t, conj v0, complex alpha/beta, a shifted window in t
    pr = sb.basic_partitioning("tNSns", dr, [n, 1, 1, 1, 1], "t", n, 1)
    vr = scatter(sb, gr, dr, pr, rank, 1, dev)
    alpha, beta = 0.5 - 1j, -1 + 0.25j
    sb.contraction(alpha, p0, [1, 0, 0, 0, 0, 0, 0], d0, d0, "tnsxyzc", True, v0, p1,
                   [1, 0, 0, 0, 0, 0, 0], d0, d0, "tNSxyzc", False, v1, beta, pr,
                   [2, 0, 0, 0, 0], dr, dr, "tNSns", vr, comm=comm)
    torch.cuda.synchronize()
    out = gather(np.zeros_like(gr), dr, pr, 1, vr)
    ref = gr.copy()
    oracle_contraction(alpha, "tnsxyzc", [1, 0, 0, 0, 0, 0, 0], d0, d0, True, g0, "tNSxyzc",
                       [1, 0, 0, 0, 0, 0, 0], d0, d0, False, g1, beta, "tNSns", [2, 0, 0, 0, 0],
                       dr, dr, ref)
    assert np.array_equal(out, ref), "contraction (b)"


def case_bsr(sb, comm, rank, n, dev, ncols=3):
    L = 4
    Lt = 2 * n
    dim = [L, L, L, Lt, 1, 3]
    b = 3
    pi = sb.basic_partitioning("xyztsc", dim, [1, 1, 1, n, 1, 1], "xyzt", n, 1)
    # domain partition: image plus a one-site halo in every lattice direction (bsr.cpp:61-79)
    pd = []
    for f, s in pi:
        f, s = list(f), list(s)
        for d in range(4):
            s[d] = min(dim[d], s[d] + 2)
            f[d] = (f[d] - 1) % dim[d] if s[d] < dim[d] else 0
        pd.append((f, s))
    f, s = pi[rank]
    sites = np.array(np.unravel_index(np.arange(vol(s[:4])), s[:4])).T + np.array(f[:4])
    dom = np.array(dim[:4])
    jj, rows = [], []
    for st in sites:
        for k, (d, dr) in enumerate([(None, 0)] + [(d, dr) for d in range(4) for dr in (-1, 1)]):
            c = st.copy()
            if d is not None:
                c[d] += dr
            jj.append(list((c - np.array(pd[rank][0][:4])) % dom) + [0, 0])
    gsite = np.ravel_multi_index(tuple((sites % dom).T), dim[:4])
    allv = gen("int", vol(dim[:4]) * 9 * b * b, 4, np.complex128).reshape(-1, 9 * b * b)
    vals = np.ascontiguousarray(allv[gsite]).ravel()
    ii = np.full(len(sites), 9, np.int32)
    op = sb.create_bsr(pi, dim, pd, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                       [torch.from_numpy(ii).to(dev)],
                       [torch.from_numpy(np.array(jj, np.int32).ravel()).to(dev)],
                       [torch.from_numpy(vals).to(dev)], comm=comm)
    dimx = [1, L, L, L, Lt, 1, 3, ncols]
    px = sb.basic_partitioning("pXYZTSCn", dimx, [1, 1, 1, 1, n, 1, 1, 1], "XYZT", n, 1)
    gx = gen("int", vol(dimx), 5, np.complex128)
    gy = gen("int", vol(dimx), 6, np.complex128)
    vx = scatter(sb, gx, dimx, px, rank, 1, dev)
    vy = scatter(sb, gy, dimx, px, rank, 1, dev)
    z8 = [0] * 8
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", z8, dimx, dimx, vx, 0.0, px,
                  "pxyztscn", z8, dimx, dimx, "p", vy, comm=comm)
    torch.cuda.synchronize()
    op.destroy()
    out = gather(np.zeros_like(gy), dimx, px, 1, vy)
    # oracle on the whole lattice: the same operator in one component
    allsites = np.array(np.unravel_index(np.arange(vol(dim[:4])), dim[:4])).T
    jg = []
    for st in allsites:
        for d, dr in [(None, 0)] + [(d, dr) for d in range(4) for dr in (-1, 1)]:
            c = st.copy()
            if d is not None:
                c[d] += dr
            jg.append(list(c % dom) + [0, 0])
    ref = np.zeros_like(gy)
    V = vol(dim[:4])
    oracle_bsr(T_CDOUBLE, dim, 0, V, b, b, np.full(V, 9, np.int32),
               np.array(jg, np.int32).ravel(), allv.ravel(), False, gx, ncols, True, ref, ncols,
               True, ncols, 1.0)
    assert np.array_equal(out, ref), "bsr"
    # powers: the second power needs the first one's halo from the neighbouring ranks
    vx = scatter(sb, gx, dimx, px, rank, 1, dev)
    dimy2 = [2] + dimx[1:]
    py2 = sb.basic_partitioning("pxyztscn", dimy2, [1, 1, 1, 1, n, 1, 1, 1], "xyzt", n, 1)
    gy2 = np.zeros(vol(dimy2), np.complex128)
    vy2 = scatter(sb, gy2, dimy2, py2, rank, 1, dev)
    op = sb.create_bsr(pi, dim, pd, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                       [torch.from_numpy(ii).to(dev)],
                       [torch.from_numpy(np.array(jj, np.int32).ravel()).to(dev)],
                       [torch.from_numpy(vals).to(dev)], comm=comm)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", z8, dimx, dimx, vx, 0.0, py2,
                  "pxyztscn", z8, dimy2, dimy2, "p", vy2, comm=comm)
    torch.cuda.synchronize()
    op.destroy()
    out2 = gather(gy2, dimy2, py2, 1, vy2)
    ref2 = np.zeros_like(ref)
    oracle_bsr(T_CDOUBLE, dim, 0, V, b, b, np.full(V, 9, np.int32),
               np.array(jg, np.int32).ravel(), allv.ravel(), False, ref, ncols, True, ref2, ncols,
               True, ncols, 1.0)
    assert np.array_equal(out2, np.concatenate([ref, ref2])), "bsr powers"
    # image side: y (domain labels) = A^H x (image labels); the halo contributions of every rank
    # are summed into their owners
    from _common import oracle_bsr_adjoint
    op = sb.create_bsr(pi, dim, pd, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                       [torch.from_numpy(ii).to(dev)],
                       [torch.from_numpy(np.array(jj, np.int32).ravel()).to(dev)],
                       [torch.from_numpy(vals).to(dev)], comm=comm)
    vx = scatter(sb, gx, dimx, px, rank, 1, dev)
    vy = scatter(sb, gy, dimx, px, rank, 1, dev)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pxyztscn", z8, dimx, dimx, vx, 0.0, px,
                  "pXYZTSCn", z8, dimx, dimx, None, vy, comm=comm)
    torch.cuda.synchronize()
    op.destroy()
    out3 = gather(np.zeros_like(gy), dimx, px, 1, vy)
    ref3 = np.zeros_like(gy)
    oracle_bsr_adjoint(T_CDOUBLE, dim, 0, V, b, b, np.full(V, 9, np.int32),
                       np.array(jg, np.int32).ravel(), allv.ravel(), False, gx, ncols, True, ref3,
                       ncols, True, V * b, ncols, 1.0)
    assert np.array_equal(out3, ref3), "bsr image side"


def case_kron(sb, comm, rank, n, dev, ncols=2, power=2):
    L, Lt, spin, color = 4, 2 * n, 4, 3
    dim = [L, L, L, Lt, spin, color]
    pi = sb.basic_partitioning("xyztsc", dim, [1, 1, 1, n, 1, 1], "xyzt", n, 1)
    pd = []
    for f, s in pi:
        f, s = list(f), list(s)
        for d in range(4):
            s[d] = min(dim[d], s[d] + 2)
            f[d] = (f[d] - 1) % dim[d] if s[d] < dim[d] else 0
        pd.append((f, s))
    f, s = pi[rank]
    sites = np.array(np.unravel_index(np.arange(vol(s[:4])), s[:4])).T + np.array(f[:4])
    dom = np.array(dim[:4])
    dirs = [(None, 0)] + [(d, dr) for d in range(4) for dr in (-1, 1)]
    jj = []
    for st in sites:
        for d, dr in dirs:
            c = st.copy()
            if d is not None:
                c[d] += dr
            jj.append(list((c - np.array(pd[rank][0][:4])) % dom) + [0, 0])
    gsite = np.ravel_multi_index(tuple((sites % dom).T), dim[:4])
    nb = color * color
    allv = gen("int", vol(dim[:4]) * 9 * nb, 4, np.complex128).reshape(-1, 9 * nb)
    vals = np.ascontiguousarray(allv[gsite]).ravel()
    kron = gen("int", 9 * spin * spin, 7, np.complex128)
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    op = sb.create_kron_bsr(pi, dim, pd, dim, blk, blk, kr, kr, False,
                            [torch.from_numpy(np.full(len(sites), 9, np.int32)).to(dev)],
                            [torch.from_numpy(np.array(jj, np.int32).ravel()).to(dev)],
                            [torch.from_numpy(vals).to(dev)], [torch.from_numpy(kron).to(dev)],
                            comm=comm)
    dimx = [1, L, L, L, Lt, color, ncols, spin]
    dimy = [power] + dimx[1:]
    px = sb.basic_partitioning("pXYZTCnS", dimx, [1, 1, 1, 1, n, 1, 1, 1], "XYZT", n, 1)
    py = sb.basic_partitioning("pxyztcns", dimy, [1, 1, 1, 1, n, 1, 1, 1], "xyzt", n, 1)
    gx = gen("int", vol(dimx), 5, np.complex128)
    gy = gen("int", vol(dimy), 6, np.complex128)
    vx = scatter(sb, gx, dimx, px, rank, 1, dev)
    vy = scatter(sb, gy, dimy, py, rank, 1, dev)
    z8 = [0] * 8
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTCnS", z8, dimx, dimx, vx, 0.0, py,
                  "pxyztcns", z8, dimy, dimy, "p", vy, comm=comm)
    torch.cuda.synchronize()
    op.destroy()
    out = gather(np.zeros_like(gy), dimy, py, 1, vy)
    allsites = np.array(np.unravel_index(np.arange(vol(dim[:4])), dim[:4])).T
    jg = []
    for st in allsites:
        for d, dr in dirs:
            c = st.copy()
            if d is not None:
                c[d] += dr
            jg.append(list(c % dom) + [0, 0])
    V = vol(dim[:4])
    cur, refs = gx, []
    for _ in range(power):
        y = np.zeros_like(cur)
        oracle_kron_bsr(T_CDOUBLE, dim[:4] + [1, 1], 0, V, 9, color, color, spin, spin,
                        np.array(jg, np.int32).ravel(), allv.ravel(), kron, False, cur, y, ncols,
                        1.0)
        refs.append(y)
        cur = y
    assert np.array_equal(out, np.concatenate(refs)), "kron bsr"


def case_dense(sb, comm, rank, n, dev):
    """cholesky / gesm / trsm with the matrices split over ranks along a row label (the working
    copy gathers whole matrices: a redistribution), and the batch label split too; with every
    dense.wave setting (2: the wave kernels for the triangular solves too, the default; 1: for
    the factorizations only; 0: the workgroup-per-matrix kernels), set alike on every rank"""
    old = sb.tune_get("dense.wave")
    try:
        for wave in (2, 1, 0):
            sb.tune_set("dense.wave", wave)
            _case_dense(sb, comm, rank, n, dev)
    finally:
        sb.tune_set("dense.wave", old)


def _case_dense(sb, comm, rank, n, dev):
    from _common import oracle_getrf, oracle_getrs, oracle_potrf
    from _dense import dense_input, from_matrices, to_matrices, to_panel, from_panel
    nt, ni = 4, 6
    dim = [nt, ni, ni]
    p = sb.basic_partitioning("tij", dim, [1, n, 1], "i", n, 1)  # rows split over ranks
    a = dense_input("hpd", nt, ni, np.complex128)
    g = from_matrices(a, "tij", dim, "i", "j")
    v = scatter(sb, g, dim, p, rank, 1, dev)
    sb.cholesky(p, dim, "tij", v, "i", "j", comm=comm)
    torch.cuda.synchronize()
    out = gather(np.zeros_like(g), dim, p, 1, v)
    w = np.ascontiguousarray(a.transpose(0, 2, 1)).ravel()
    assert oracle_potrf(w, ni, nt) == 0
    ref = from_matrices(w.reshape(nt, ni, ni).transpose(0, 2, 1), "tij", dim, "i", "j")
    assert np.allclose(out, ref, rtol=0, atol=1e-12 * np.abs(ref).max()), "dense cholesky"
    # gesm: C split over t, x (another label order) split over t too -- the right-hand-side
    # labels of x must be whole in each component, as in the reference (dense.h:565-598) --,
    # y split over its rows
    c = dense_input("gen", nt, ni, np.complex128)
    gc = from_matrices(c, "tij", dim, "i", "j")
    pc = sb.basic_partitioning("tij", dim, [n, 1, 1], "t", n, 1)
    dimx = [nt, ni, 4]
    dimxp = [4, nt, ni]  # "ntj"
    px = sb.basic_partitioning("ntj", dimxp, [1, n, 1], "t", n, 1)
    py = sb.basic_partitioning("tin", dimx, [1, n, 1], "i", n, 1)
    gx = gen("int", vol(dimx), 5, np.complex128)
    gxp = np.ascontiguousarray(gx.reshape(dimx).transpose(2, 0, 1)).ravel()
    vc = scatter(sb, gc, dim, pc, rank, 1, dev)
    vx = scatter(sb, gxp, dimxp, px, rank, 1, dev)
    vy = scatter(sb, np.zeros_like(gx), dimx, py, rank, 1, dev)
    sb.gesm(2.0, pc, dim, "tij", vc, "i", "j", px, dimxp, "ntj", vx, py, dimx, "tin", vy,
            comm=comm)
    torch.cuda.synchronize()
    out = gather(np.zeros_like(gx), dimx, py, 1, vy)
    w = np.ascontiguousarray(c.transpose(0, 2, 1)).ravel()
    piv = np.zeros(nt * ni, np.int32)
    assert oracle_getrf(w, ni, nt, piv) == 0
    xm = np.ascontiguousarray(to_panel(gx, "tjn", dimx, "n", "j")).ravel()
    oracle_getrs(w, ni, nt, piv, 4, xm)
    ref = 2.0 * from_panel(xm.reshape(nt, 4, ni), "tin", dimx, "n", "i")
    assert np.allclose(out, ref, rtol=0, atol=1e-12 * np.abs(ref).max()), "dense gesm"
    # trsm: an upper triangular C (its strict lower part is garbage the solve must not read)
    # split over t, x over t, y over its rows
    ct = dense_input("tri", nt, ni, np.complex128)
    vc = scatter(sb, from_matrices(ct, "tij", dim, "i", "j"), dim, pc, rank, 1, dev)
    vy = scatter(sb, np.zeros_like(gx), dimx, py, rank, 1, dev)
    sb.trsm(0.5 - 1j, pc, dim, "tij", vc, "i", "j", px, dimxp, "ntj", vx, py, dimx, "tin", vy,
            comm=comm)
    torch.cuda.synchronize()
    out = gather(np.zeros_like(gx), dimx, py, 1, vy)
    xs = gx.reshape(dimx)
    ref = np.stack([(0.5 - 1j) * np.linalg.solve(np.triu(ct[t]), xs[t]) for t in range(nt)]).ravel()
    assert np.allclose(out, ref, rtol=0, atol=1e-12 * np.abs(ref).max()), "dense trsm"


def case_storage(sb, comm, rank, n, dev):
    from oracle import s3t
    dim = [6, 5, 5]  # storage "abc"
    dim0 = [5, 6, 5]  # tensor "cab", split over a
    p0 = sb.basic_partitioning("cab", dim0, [1, n, 1], "a", n, 1)
    g0 = gen("index", vol(dim0), 1, np.complex128)
    blocks = [([0, 0, 0], [3, 5, 5]), ([3, 1, 0], [3, 2, 5]), ([3, 4, 0], [3, 2, 5])]  # wraps b
    stored = np.zeros(dim, bool)
    stored[0:3] = True
    stored[3:6, [1, 2, 4, 0]] = True  # b = 3 is never stored for a >= 3
    S = (2.0 - 1.0j) * g0.reshape(dim0).transpose(1, 2, 0)  # S[a, b, c] = alpha * v0[c, a, b]
    fn = os.path.join("/tmp", "sbx_dist_storage_%s.s3t" % os.environ.get("MASTER_PORT", "0"))
    for checksum in (sb.GlobalChecksum, sb.BlockChecksum):
        sto = sb.create_storage(dim, sb.SlowToFast, fn, b"dist", checksum, torch.complex128,
                                comm=comm)
        sb.append_blocks(sto, blocks, dim, comm=comm)
        v0 = scatter(sb, g0, dim0, p0, rank, 1, dev)
        sb.save(2.0 - 1.0j, p0, "cab", [0, 0, 0], dim0, dim0, v0, "abc", [0, 0, 0], sto,
                comm=comm)
        sto.close(comm)
        if rank == 0:
            with open(fn, "rb") as f:
                st = s3t.parse(f.read())  # verifies every checksum
            got = [(b["from"], b["size"]) for ch in st["chunks"] for b in ch]
            assert got == [(list(f), list(sz)) for f, sz in blocks], ("storage blocks", got)
            for ch in st["chunks"]:
                for b in ch:
                    assert np.array_equal(b["values"], piece(S.ravel(), dim, b["from"],
                                                             b["size"])), "storage values"
        dist.barrier()
        # load back into "bca" split over c, with the unstored elements untouched
        diml = [5, 5, 6]
        pl = sb.basic_partitioning("bca", diml, [1, n, 1], "c", n, 1)
        gl = gen("int", vol(diml), 2, np.complex128)
        vl = scatter(sb, gl, diml, pl, rank, 1, dev)
        sto = sb.open_storage(fn, False, comm=comm)
        sb.check_storage(sto, comm)
        sb.load(1.0, sto, "abc", [0, 0, 0], dim, pl, "bca", [0, 0, 0], diml, vl, comm=comm)
        torch.cuda.synchronize()
        sto.close(comm)
        out = gather(np.zeros_like(gl), diml, pl, 1, vl)
        ref = np.where(stored.transpose(1, 2, 0), S.transpose(1, 2, 0),
                       gl.reshape(diml)).ravel()
        assert np.array_equal(out, ref), "storage load"
        dist.barrier()
    if rank == 0:
        os.remove(fn)


def case_split(sb, comm, rank, n, dev, ncols=3):
    """The reference's split operator (tests/bsr.cpp:402-545, 779-818): the 9-point operator as a
    core piece (domain = the rank's own sites, no exchange, applied with just_local) plus a halo
    piece (the blocks reaching other ranks' sites, domain = image + halo).  The halo piece is
    applied first with a deferred request (its exchange in flight), the core piece runs, then
    the request is waited: y = core x + halo x must equal the whole operator's product."""
    L = 4
    Lt = 2 * n
    dim = [L, L, L, Lt, 1, 3]
    b = 3
    pi = sb.basic_partitioning("xyztsc", dim, [1, 1, 1, n, 1, 1], "xyzt", n, 1)
    pd = []
    for f, s in pi:
        f, s = list(f), list(s)
        for d in range(4):
            s[d] = min(dim[d], s[d] + 2)
            f[d] = (f[d] - 1) % dim[d] if s[d] < dim[d] else 0
        pd.append((f, s))
    f, s = pi[rank]
    sites = np.array(np.unravel_index(np.arange(vol(s[:4])), s[:4])).T + np.array(f[:4])
    dom = np.array(dim[:4])
    lo, sz = np.array(f[:4]), np.array(s[:4])
    jj_core, jj_halo = [], []
    for st in sites:
        for d, dr in [(None, 0)] + [(d, dr) for d in range(4) for dr in (-1, 1)]:
            c = st.copy()
            if d is not None:
                c[d] += dr
            inside = np.all((c - lo) % dom < sz)
            jj_core.append(list((c - lo) % dom) + [0, 0] if inside else [-1] * 6)
            jj_halo.append([-1] * 6 if inside else list((c - np.array(pd[rank][0][:4])) % dom)
                           + [0, 0])
    gsite = np.ravel_multi_index(tuple((sites % dom).T), dim[:4])
    allv = gen("int", vol(dim[:4]) * 9 * b * b, 4, np.complex128).reshape(-1, 9 * b * b)
    vals = torch.from_numpy(np.ascontiguousarray(allv[gsite]).ravel()).to(dev)
    ii = torch.from_numpy(np.full(len(sites), 9, np.int32)).to(dev)
    blk = [1, 1, 1, 1, 1, 3]
    core = sb.create_bsr(pi, dim, pi, dim, blk, blk, False, [ii],
                         [torch.from_numpy(np.array(jj_core, np.int32).ravel()).to(dev)], [vals],
                         comm=comm)
    halo = sb.create_bsr(pi, dim, pd, dim, blk, blk, False, [ii],
                         [torch.from_numpy(np.array(jj_halo, np.int32).ravel()).to(dev)], [vals],
                         comm=comm)
    dimx = [1, L, L, L, Lt, 1, 3, ncols]
    px = sb.basic_partitioning("pXYZTSCn", dimx, [1, 1, 1, 1, n, 1, 1, 1], "XYZT", n, 1)
    gx = gen("int", vol(dimx), 5, np.complex128)
    vx = scatter(sb, gx, dimx, px, rank, 1, dev)
    vy = scatter(sb, np.zeros(vol(dimx), np.complex128), dimx, px, rank, 1, dev)
    z8 = [0] * 8
    req = sb.bsr_krylov(1.0, halo, "xyztsc", "XYZTSC", px, "pXYZTSCn", z8, dimx, dimx, vx, 1.0,
                        px, "pxyztscn", z8, dimx, dimx, "p", vy, comm=comm, request=True)
    assert req is not None, "the halo piece's exchange should be left in flight"
    assert sb.bsr_krylov(1.0, core, "xyztsc", "XYZTSC", px, "pXYZTSCn", z8, dimx, dimx, vx, 1.0,
                         px, "pxyztscn", z8, dimx, dimx, "p", vy, comm=comm, request=True,
                         just_local=True) is None
    req.wait()
    torch.cuda.synchronize()
    core.destroy()
    halo.destroy()
    out = gather(np.zeros(vol(dimx), np.complex128), dimx, px, 1, vy)
    allsites = np.array(np.unravel_index(np.arange(vol(dim[:4])), dim[:4])).T
    jg = []
    for st in allsites:
        for d, dr in [(None, 0)] + [(d, dr) for d in range(4) for dr in (-1, 1)]:
            c = st.copy()
            if d is not None:
                c[d] += dr
            jg.append(list(c % dom) + [0, 0])
    ref = np.zeros(vol(dimx), np.complex128)
    V = vol(dim[:4])
    oracle_bsr(T_CDOUBLE, dim, 0, V, b, b, np.full(V, 9, np.int32), np.array(jg, np.int32).ravel(),
               allv.ravel(), False, gx, ncols, True, ref, ncols, True, ncols, 1.0)
    assert np.array_equal(out, ref), "split operator"
    # a deferred distributed copy: the exchange in flight, finished by wait()
    dim0, dim1 = [4, 4, 2, 2 * n], [2 * n, 2, 4, 4]
    p0 = sb.basic_partitioning("xyzt", dim0, [1, 1, 1, n], "t", n, 1)
    p1 = sb.basic_partitioning("tzyx", dim1, [1, 1, 1, n], "x", n, 1)
    g0 = gen("index", vol(dim0), 1, np.complex128)
    g1 = gen("int", vol(dim1), 2, np.complex128)
    v0 = scatter(sb, g0, dim0, p0, rank, 1, dev)
    v1 = scatter(sb, g1, dim1, p1, rank, 1, dev)
    r = sb.copy(1.0, p0, "xyzt", [0] * 4, dim0, dim0, v0, p1, "tzyx", [0] * 4, dim1, v1,
                comm=comm, request=True)
    sb.wait(r)
    torch.cuda.synchronize()
    out = gather(np.zeros_like(g1), dim1, p1, 1, v1)
    ref = g1.copy()
    oracle_copy(1.0, "xyzt", [0] * 4, dim0, dim0, g0, "tzyx", [0] * 4, dim1, ref)
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8)), "deferred copy"


LATTICE_GRID = {1: [1, 1, 1], 2: [2, 1, 1], 3: [3, 1, 1], 4: [2, 2, 1], 8: [2, 2, 2]}


def case_reduce(sb, comm, rank, n, dev, transport):
    """The contraction's partial outputs summed by one RCCL collective (ncclReduce into an owner,
    ncclAllReduce into a replicated output) and by the point-to-point Add copy (dist.reduce 0):
    both exact against the oracle on integer data, and the collective is what runs with RCCL."""
    L, nn = 4, 2
    d0 = [L, nn, 4, L, L, L * n, 3]
    dr = [L, nn, 4, nn, 4]
    p0 = sb.basic_partitioning("tnsxyzc", d0, [1, 1, 1, 1, 1, n, 1], "z", n, 1)
    g0 = gen("int", vol(d0), 11, np.complex128)
    g1 = gen("int", vol(d0), 12, np.complex128)
    gr = gen("int", vol(dr), 13, np.complex128)
    v0 = scatter(sb, g0, d0, p0, rank, 1, dev)
    v1 = scatter(sb, g1, d0, p0, rank, 1, dev)
    z7, z5 = [0] * 7, [0] * 5
    alpha, beta = 2 - 1j, 0.5 + 1j
    ref = gr.copy()
    oracle_contraction(alpha, "tnsxyzc", z7, d0, d0, False, g0, "tNSxyzc", z7, d0, d0, True, g1,
                       beta, "tNSns", z5, dr, dr, ref)
    owner = n - 1  # not rank 0
    outputs = {
        "owner": [([0] * 5, dr if q == owner else [0] * 5) for q in range(n)],
        "replicated": [([0] * 5, dr)] * n,
    }
    for mode in (1, 0):
        sb.tune_set("dist.reduce", mode)
        try:
            for name, pr in outputs.items():
                vr = scatter(sb, gr, dr, pr, rank, 1, dev)
                if vr[0].numel() == 0:
                    vr = [torch.zeros(1, dtype=torch.complex128, device=dev)]
                sb.tune_set("dist.reduce_calls", 0)
                sb.contraction(alpha, p0, z7, d0, d0, "tnsxyzc", False, v0, p0, z7, d0, d0,
                               "tNSxyzc", True, v1, beta, pr, z5, dr, dr, "tNSns", vr, comm=comm)
                torch.cuda.synchronize()
                calls = sb.tune_get("dist.reduce_calls")
                if transport == "rccl" and mode == 1:
                    assert calls > 0, ("collective reduce not used", name)
                else:
                    assert calls == 0, ("collective reduce used", name, mode, transport)
                if name == "replicated" or rank == owner:
                    assert np.array_equal(vr[0].cpu().numpy(), ref), ("reduce", name, mode)
        finally:
            sb.tune_set("dist.reduce", 1)


def case_golden(sb, comm, rank, n, dev):
    grid = LATTICE_GRID.get(n, [n, 1, 1])
    for case in manifest("contraction"):
        if (case.get("gen", "int") == "int" or case["o0"] != "tnsxyzc" or len(case["p0"]) != 1
                or case["t"] != "cdouble"):
            continue
        g0, g1, gr = contraction_inputs(case)
        d0, d1, dr = case["dim0"], case["dim1"], case["dimr"]
        p0 = sb.basic_partitioning("tnsxyzc", d0, [1, 1, 1] + grid + [1], "xyz", n, 1)
        for shape in ("4a", "4b"):
            if shape == "4a":
                p1 = sb.basic_partitioning(case["o1"], d1, [1, 1, 1] + grid + [1], "xyz", n, 1)
            else:
                p1 = sb.basic_partitioning(case["o1"], d1, [n, 1, 1, 1, 1, 1, 1], "t", n, 1)
            pr = [([0] * len(dr), dr)] + [([0] * len(dr), [0] * len(dr))] * (n - 1)
            v0 = scatter(sb, g0, d0, p0, rank, 1, dev)
            v1 = scatter(sb, g1, d1, p1, rank, 1, dev)
            vr = scatter(sb, gr, dr, pr, rank, 1, dev)
            if vr[0].numel() == 0:
                vr = [torch.zeros(1, dtype=torch.complex128, device=dev)]
            beta = complex(*case["beta"])
            for mode in (1, 0):  # RCCL collective reduction / point-to-point Add copy
                sb.tune_set("dist.reduce", mode)
                vr = scatter(sb, gr, dr, pr, rank, 1, dev)
                if vr[0].numel() == 0:
                    vr = [torch.zeros(1, dtype=torch.complex128, device=dev)]
                try:
                    sb.contraction(complex(*case["alpha"]), p0, case["from0"], case["size0"], d0,
                                   case["o0"], case["conj0"], v0, p1, case["from1"],
                                   case["size1"], d1, case["o1"], case["conj1"], v1, beta, pr,
                                   case["fromr"], case["sizer"], dr, case["o_r"], vr, comm=comm)
                finally:
                    sb.tune_set("dist.reduce", 1)
                torch.cuda.synchronize()
                out = gather(np.zeros_like(gr), dr, pr, 1, vr[:1] if rank == 0 else [vr[0][:0]])
                errs = component_errors(out, output(case, np.complex128))
                assert max(errs) < 1e-10, ("golden", case["id"], shape, mode, errs)


def case_debug(sb, comm, rank, n, dev):
    """SB_DEBUG (tune key debug.level): at 2 the distributed copies run the mock-index check
    (dist.h:1919-2116) on every rank; at 1 a rank called with different arguments makes EVERY
    rank fail (check_consistency, dist.h:702-736) instead of leaving the others in an exchange"""
    old = sb.tune_get("debug.level")
    try:
        sb.tune_set("debug.level", 2)
        case_copy(sb, comm, rank, n, dev)
        case_fuzz(sb, comm, rank, n, dev, ncases=4)
        sb.tune_set("debug.level", 1)
        dim0, dim1 = [4, 4, 2, 6], [6, 2, 4, 4]
        p0 = sb.basic_partitioning("xyzt", dim0, [1, 1, 1, n], "t", n, 1)
        p1 = sb.basic_partitioning("tzyx", dim1, [1, 1, 1, n], "x", n, 1)
        v0 = scatter(sb, gen("index", vol(dim0), 1, np.complex128), dim0, p0, rank, 1, dev)
        v1 = scatter(sb, gen("int", vol(dim1), 2, np.complex128), dim1, p1, rank, 1, dev)
        try:
            sb.copy(2.0 if rank == n - 1 else 1.0, p0, "xyzt", [0] * 4, dim0, dim0, v0, p1,
                    "tzyx", [0] * 4, dim1, v1, comm=comm)
        except sb.SuperbblasError as e:
            assert "check_consistency failed" in str(e), e
        else:
            raise AssertionError("check_consistency missed different arguments on rank %d" % rank)
        # the same call with equal arguments still works afterwards
        sb.copy(1.0, p0, "xyzt", [0] * 4, dim0, dim0, v0, p1, "tzyx", [0] * 4, dim1, v1, comm=comm)
        torch.cuda.synchronize()
        # at 2 a wrong plan on ONE rank (debug.corrupt_copy drops its first local piece) makes
        # EVERY rank fail the mock-index check, so no rank is left waiting in the real copy's
        # exchange; the library is usable afterwards
        sb.tune_set("debug.level", 2)
        if rank == 0:
            sb.tune_set("debug.corrupt_copy", 1)
        try:
            sb.copy(1.0, p0, "xyzt", [0] * 4, dim0, dim0, v0, p1, "tzyx", [0] * 4, dim1, v1,
                    comm=comm)
        except sb.SuperbblasError as e:
            assert "test_copy_check does not pass" in str(e), e
        else:
            raise AssertionError("the mock-index check let a corrupt copy through on rank %d" % rank)
        finally:
            sb.tune_set("debug.corrupt_copy", 0)
        sb.copy(1.0, p0, "xyzt", [0] * 4, dim0, dim0, v0, p1, "tzyx", [0] * 4, dim1, v1, comm=comm)
        torch.cuda.synchronize()
    finally:
        sb.tune_set("debug.level", old)


def case_peer(sb, comm, rank, n, dev):
    nc = 2
    sb.tune_set("dist.force_peer", 1)
    sb.tune_set("dist.peer_copies", 0)
    try:
        dim0, dim1 = [4, 4, 2, 6], [6, 2, 4, 4]
        p0 = sb.basic_partitioning("xyzt", dim0, [1, 1, 1, n], "t", n, nc)
        p1 = sb.basic_partitioning("tzyx", dim1, [1, 1, 1, n], "x", n, nc)
        g0 = gen("index", vol(dim0), 1, np.complex128)
        for add in (False, True):
            g1 = gen("int", vol(dim1), 2, np.complex128)
            v0 = _nonempty(scatter(sb, g0, dim0, p0, rank, nc, dev), dev)
            v1 = _nonempty(scatter(sb, g1, dim1, p1, rank, nc, dev), dev)
            sb.copy(2.0 if add else 1.0, p0, "xyzt", [1, 2, 0, 3], [3, 4, 2, 5], dim0, v0, p1,
                    "tzyx", [2, 0, 1, 3], dim1, v1, copyadd=sb.Add if add else sb.Copy, comm=comm)
            torch.cuda.synchronize()
            out = gather(np.zeros_like(g1), dim1, p1, nc,
                         [v1[i][:vol(p1[rank * nc + i][1])] for i in range(nc)])
            ref = g1.copy()
            oracle_copy(2.0 if add else 1.0, "xyzt", [1, 2, 0, 3], [3, 4, 2, 5], dim0, g0, "tzyx",
                        [2, 0, 1, 3], dim1, ref, add=add)
            assert np.array_equal(out.view(np.uint8), ref.view(np.uint8)), ("peer copy", add)
        grid = LATTICE_GRID.get(n, [n, 1, 1])
        for case in manifest("contraction"):
            if (case.get("gen", "int") == "int" or case["o0"] != "tnsxyzc" or len(case["p0"]) != 1
                    or case["t"] != "cdouble"):
                continue
            g0, g1, gr = contraction_inputs(case)
            d0, d1, dr = case["dim0"], case["dim1"], case["dimr"]
            p0 = sb.basic_partitioning("tnsxyzc", d0, [1, 1, 1] + grid + [1], "xyz", n, nc)
            p1 = sb.basic_partitioning(case["o1"], d1, [n, 1, 1, 1, 1, 1, 1], "t", n, nc)
            pr = [([0] * len(dr), dr)] + [([0] * len(dr), [0] * len(dr))] * (n * nc - 1)
            v0 = _nonempty(scatter(sb, g0, d0, p0, rank, nc, dev), dev)
            v1 = _nonempty(scatter(sb, g1, d1, p1, rank, nc, dev), dev)
            vr = _nonempty(scatter(sb, gr, dr, pr, rank, nc, dev), dev)
            sb.contraction(complex(*case["alpha"]), p0, case["from0"], case["size0"], d0,
                           case["o0"], case["conj0"], v0, p1, case["from1"], case["size1"], d1,
                           case["o1"], case["conj1"], v1, complex(*case["beta"]), pr,
                           case["fromr"], case["sizer"], dr, case["o_r"], vr, comm=comm)
            torch.cuda.synchronize()
            out = gather(np.zeros_like(gr), dr, pr, nc,
                         [vr[i][:vol(pr[rank * nc + i][1])] for i in range(nc)])
            errs = component_errors(out, output(case, np.complex128))
            assert max(errs) < 1e-10, ("peer golden", case["id"], errs)
        assert sb.tune_get("dist.peer_copies") > 0, "the peer path did not run"
    finally:
        sb.tune_set("dist.force_peer", 0)


def _rand_partition(sb, rng, labels, dims, n):
    i = int(rng.integers(0, len(dims)))
    procs = [1] * len(dims)
    procs[i] = n
    return sb.basic_partitioning(labels, dims, procs, labels[i], n, 1)


def _nonempty(ts, dev):
    """A rank that owns no element still passes a valid (1-element) buffer."""
    return [t if t.numel() else torch.zeros(1, dtype=t.dtype, device=dev) for t in ts]


def case_fuzz(sb, comm, rank, n, dev, ncases=12, big=False):
    """big: extents to 16 (operands to ~64K elements), so the pieces exchanged take the
    transpose / tile kernels and the contractions the matrix-core GEMM forms"""
    letters = "abcdefgh"

    def extent(rng):
        return int(rng.choice([1, 2, 3, 4, 6, 8, 12, 16])) if big else int(rng.integers(1, 6))

    for seed in range(ncases):
        rng = np.random.default_rng((4242 if big else 777) + seed)
        # copy
        nd = int(rng.integers(1, 6))
        o0 = "".join(rng.permutation(list(letters))[:nd])
        o1 = "".join(rng.permutation(list(o0)))
        while True:
            ext = {c: extent(rng) for c in o0}
            if vol(ext.values()) <= 1 << 16:
                break
        d0, d1 = [ext[c] for c in o0], [ext[c] for c in o1]
        f0 = [int(rng.integers(0, d)) for d in d0]
        s0 = [int(rng.integers(1, d + 1)) for d in d0]
        f1 = [int(rng.integers(0, d)) for d in d1]
        t0, t1 = [(np.complex128, np.complex128), (np.complex64, np.complex128),
                  (np.float64, np.complex128)][int(rng.integers(0, 3))]
        add = bool(rng.integers(0, 2))
        p0 = _rand_partition(sb, rng, o0, d0, n)
        p1 = _rand_partition(sb, rng, o1, d1, n)
        g0 = gen("int", vol(d0), seed, t0)
        g1 = gen("int", vol(d1), seed + 1, t1)
        v0 = _nonempty(scatter(sb, g0, d0, p0, rank, 1, dev), dev)
        v1 = _nonempty(scatter(sb, g1, d1, p1, rank, 1, dev), dev)
        sb.copy(1.0, p0, o0, f0, s0, d0, v0, p1, o1, f1, d1, v1,
                copyadd=sb.Add if add else sb.Copy, comm=comm)
        torch.cuda.synchronize()
        out = gather(np.zeros_like(g1), d1, p1, 1, [v1[0][:vol(p1[rank][1])]])
        ref = g1.copy()
        oracle_copy(1.0, o0, f0, s0, d0, g0, o1, f1, d1, ref, add=add)
        assert np.array_equal(out.view(np.uint8), ref.view(np.uint8)), ("fuzz copy", seed)
        # contraction
        cnt = [int(rng.integers(0, 3)) for _ in range(4)]
        if cnt[0] + cnt[1] + cnt[2] == 0:
            cnt[2] = 1  # every tensor has a label (a partition needs a dimension)
        if cnt[0] + cnt[1] + cnt[3] == 0:
            cnt[3] = 1
        if cnt[0] + cnt[2] + cnt[3] == 0:
            cnt[2] = 1
        ls = list(rng.permutation(list(letters)))
        T, A = "".join(ls[:cnt[0]]), "".join(ls[cnt[0]:sum(cnt[:2])])
        B, C = "".join(ls[sum(cnt[:2]):sum(cnt[:3])]), "".join(ls[sum(cnt[:3]):sum(cnt)])
        while True:
            ext = {c: (extent(rng) if big else int(rng.integers(1, 5))) for c in T + A + B + C}
            if max(vol([ext[c] for c in g]) for g in (T + A + B, T + A + C, T + B + C)) <= 1 << 16:
                break
        o0 = "".join(rng.permutation(list(T + A + B)))
        o1 = "".join(rng.permutation(list(T + A + C)))
        o_r = "".join(rng.permutation(list(T + B + C)))
        d0, d1, dr = ([ext[c] for c in o] for o in (o0, o1, o_r))
        bs = {c: int(rng.integers(1, ext[c] + 1)) if rng.random() < 0.4 else ext[c] for c in ext}
        f0 = [int(rng.integers(0, ext[c])) for c in o0]
        f1 = [int(rng.integers(0, ext[c])) for c in o1]
        fr = [int(rng.integers(0, ext[c])) for c in o_r]
        s0, s1, sr = ([bs[c] for c in o] for o in (o0, o1, o_r))
        alpha = complex(rng.uniform(-1, 1), rng.uniform(-1, 1))
        beta = [0.0, 1.0, 0.5 - 0.25j][int(rng.integers(0, 3))]
        conj0, conj1 = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        p0 = _rand_partition(sb, rng, o0, d0, n)
        p1 = _rand_partition(sb, rng, o1, d1, n)
        pr = _rand_partition(sb, rng, o_r, dr, n)
        g0 = gen("int", vol(d0), 10 + seed, np.complex128)
        g1 = gen("int", vol(d1), 20 + seed, np.complex128)
        gr = gen("int", vol(dr), 30 + seed, np.complex128)
        v0 = _nonempty(scatter(sb, g0, d0, p0, rank, 1, dev), dev)
        v1 = _nonempty(scatter(sb, g1, d1, p1, rank, 1, dev), dev)
        vr = _nonempty(scatter(sb, gr, dr, pr, rank, 1, dev), dev)
        sb.contraction(alpha, p0, f0, s0, d0, o0, conj0, v0, p1, f1, s1, d1, o1, conj1, v1, beta,
                       pr, fr, sr, dr, o_r, vr, comm=comm)
        torch.cuda.synchronize()
        out = gather(np.zeros_like(gr), dr, pr, 1, [vr[0][:vol(pr[rank][1])]])
        ref = gr.copy()
        oracle_contraction(alpha, o0, f0, s0, d0, conj0, g0, o1, f1, s1, d1, conj1, g1, beta, o_r,
                           fr, sr, dr, ref)
        assert rel_err(out, ref) < 1e-10, ("fuzz contraction", seed, o0, o1, o_r, d0, d1, dr)


def main():
    transport = os.environ.get("SBX_TEST_TRANSPORT", "host")
    if transport == "rccl" and os.environ.get("SBX_RCCL_SHARED_GPU") == "1":
        # several RCCL ranks on one GPU (a 1-GPU test box): RCCL refuses two ranks of one host on
        # one device, so every rank declares its own host id; the ranks then exchange through
        # RCCL's network transport over loopback sockets.  The library's RCCL code path (grouped
        # ncclSend/ncclRecv on its streams, the side-stream pipeline) is the one that runs.
        os.environ["NCCL_HOSTID"] = "sbx-test-rank-%s" % os.environ.get("RANK", "0")
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    ndev = torch.cuda.device_count()
    dev_idx = int(os.environ.get("LOCAL_RANK", "0")) % ndev
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    if os.environ.get("SBX_TEST_PG") == "nccl":
        # the process group of bench.py's real N > 1 start-up: torch's own RCCL communicator,
        # created eagerly on this rank's device, beside the library's (Comm.from_torch_distributed)
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    rank, n = dist.get_rank(), dist.get_world_size()
    import superbblas_amd as sb
    if transport == "rccl":
        comm = sb.Comm.from_torch_distributed(dev_idx)
    else:
        comm = sb.Comm.host_staged(dev_idx)
    cases = os.environ.get("SBX_TEST_CASES", "copy,contr,bsr,kron,dense,storage,fuzz,fuzzl,golden,split,reduce,debug").split(",")
    if "copy" in cases:
        case_copy(sb, comm, rank, n, dev)
    if "contr" in cases:
        case_contraction(sb, comm, rank, n, dev)
    if "bsr" in cases:
        case_bsr(sb, comm, rank, n, dev)
    if "kron" in cases:
        case_kron(sb, comm, rank, n, dev)
    if "dense" in cases:
        case_dense(sb, comm, rank, n, dev)
    if "storage" in cases:
        case_storage(sb, comm, rank, n, dev)
    if "fuzz" in cases:
        case_fuzz(sb, comm, rank, n, dev)
    if "fuzzl" in cases:
        case_fuzz(sb, comm, rank, n, dev, ncases=16, big=True)
    if "golden" in cases:
        case_golden(sb, comm, rank, n, dev)
    if "reduce" in cases:
        case_reduce(sb, comm, rank, n, dev, transport)
    if "split" in cases:
        case_split(sb, comm, rank, n, dev)
    if "debug" in cases:
        case_debug(sb, comm, rank, n, dev)
    if "peer" in cases:
        case_peer(sb, comm, rank, n, dev)
    dist.barrier()
    comm.close()
    dist.destroy_process_group()
    if rank == 0:
        print("DIST OK ranks=%d transport=%s cases=%s" % (n, transport, ",".join(cases)))


if __name__ == "__main__":
    main()
