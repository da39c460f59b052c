"""Seeded random parity sweep of contraction(), copy() and bsr_krylov() on the GPU against the oracle
(oracle/oracle.c, pinned to the reference by tests/test_oracle_golden.py).

Every case draws label groups (T batch, A summed, B / C free), extents, label orders, boxes
(from/size, periodic, possibly wrapping), conjugation, alpha/beta and a split of the operands
into components, so the planner's in-place / sub-box / temporary paths and the GEMM's stride
forms are all crossed.  Bars: contraction <= 1e-10 relative (complex<double>, random values;
1e-12 double, 2e-5 single precision) and untouched elements outside the output box
bit-identical; copy and BSR bit-exact (integer-valued data)."""
import numpy as np
import pytest

from _common import int_valued, oracle_contraction, oracle_copy, random_valued, rel_err

pytestmark = pytest.mark.gpu

_LETTERS = "abcdefghij"


def _vol(d):
    n = 1
    for x in d:
        n *= x
    return n


def _split(sb, gpu, v, labels, dims, rng):
    """The tensor as 1 or 2 components (split along a random label of extent >= 2)."""
    import torch
    cand = [i for i, d in enumerate(dims) if d >= 2]
    if not cand or rng.random() < 0.5:
        return [([0] * len(dims), list(dims))], [torch.from_numpy(v.copy()).to(gpu)]
    i = int(rng.choice(cand))
    procs = [1] * len(dims)
    procs[i] = 2
    p = sb.basic_partitioning(labels, dims, procs, labels[i], 2, 1)
    full = v.reshape(dims)
    comps = []
    for frm, size in p:
        sl = tuple(slice(f, f + s) for f, s in zip(frm, size))
        comps.append(torch.from_numpy(np.ascontiguousarray(full[sl]).ravel()).to(gpu))
    return p, comps


def _gather(p, comps, dims, dtype):
    out = np.zeros(dims, dtype)
    for (frm, size), t in zip(p, comps):
        sl = tuple(slice(f, f + s) for f, s in zip(frm, size))
        out[sl] = t.cpu().numpy().reshape(size)
    return out.ravel()


def _box(rng, dims):
    frm = [int(rng.integers(0, d)) for d in dims]
    size = [int(rng.integers(1, d + 1)) if rng.random() < 0.5 else d for d in dims]
    return frm, size


@pytest.mark.parametrize("seed", range(48))
def test_fuzz_contraction(gpu, seed):
    _fuzz_contraction(gpu, seed, np.complex128, 1e-10)


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("dtype,tol", [(np.complex64, 2e-5), (np.float64, 1e-12),
                                       (np.float32, 2e-5)])
def test_fuzz_contraction_types(gpu, seed, dtype, tol):
    _fuzz_contraction(gpu, 100 + seed, dtype, tol)


def _fuzz_contraction(gpu, seed, dtype, tol):
    import torch
    import superbblas_amd as sb
    rng = np.random.default_rng(1000 + seed)
    counts = [int(rng.integers(0, 3)) for _ in range(4)]  # T, A, B, C
    if counts[0] + counts[2] + counts[3] == 0:
        counts[2] = 1
    letters = list(rng.permutation(list(_LETTERS)))
    T = "".join(letters[:counts[0]])
    A = "".join(letters[counts[0]:sum(counts[:2])])
    B = "".join(letters[sum(counts[:2]):sum(counts[:3])])
    C = "".join(letters[sum(counts[:3]):sum(counts)])
    ext = {c: int(rng.integers(1, 5)) for c in T + A + B + C}
    o0 = "".join(rng.permutation(list(T + A + B)))
    o1 = "".join(rng.permutation(list(T + A + C)))
    o_r = "".join(rng.permutation(list(T + B + C)))
    d0, d1, dr = ([ext[c] for c in o] for o in (o0, o1, o_r))
    # boxes: shared labels have the same box size; origins differ per tensor
    bsize = {c: (int(rng.integers(1, ext[c] + 1)) if rng.random() < 0.4 else ext[c]) for c in ext}
    f0 = [int(rng.integers(0, ext[c])) if bsize[c] < ext[c] or rng.random() < 0.3 else 0 for c in o0]
    f1 = [int(rng.integers(0, ext[c])) if bsize[c] < ext[c] or rng.random() < 0.3 else 0 for c in o1]
    fr = [int(rng.integers(0, ext[c])) if bsize[c] < ext[c] or rng.random() < 0.3 else 0 for c in o_r]
    s0, s1, sr = ([bsize[c] for c in o] for o in (o0, o1, o_r))
    conj0, conj1 = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
    cplx = np.dtype(dtype).kind == "c"
    alpha = complex(rng.uniform(-2, 2), rng.uniform(-2, 2)) if cplx else float(rng.uniform(-2, 2))
    beta = [0.0, 1.0, complex(rng.uniform(-1, 1), rng.uniform(-1, 1)) if cplx else
            float(rng.uniform(-1, 1))][int(rng.integers(0, 3))]
    v0 = random_valued(_vol(d0), dtype, 3 * seed + 1)
    v1 = random_valued(_vol(d1), dtype, 3 * seed + 2)
    vr = random_valued(_vol(dr), dtype, 3 * seed + 3)
    ref = vr.copy()
    oracle_contraction(alpha, o0, f0, s0, d0, conj0, v0, o1, f1, s1, d1, conj1, v1, beta, o_r,
                       fr, sr, dr, ref)
    p0, c0 = _split(sb, gpu, v0, o0, d0, rng)
    p1, c1 = _split(sb, gpu, v1, o1, d1, rng)
    pr, cr = _split(sb, gpu, vr, o_r, dr, rng)
    sb.contraction(alpha, p0, f0, s0, d0, o0, conj0, c0, p1, f1, s1, d1, o1, conj1, c1, beta, pr,
                   fr, sr, dr, o_r, cr)
    torch.cuda.synchronize()
    out = _gather(pr, cr, dr, dtype)
    case = (o0, o1, o_r, d0, d1, dr, f0, f1, fr, s0, conj0, conj1, alpha, beta)
    assert rel_err(out, ref) < tol, case
    inside = np.zeros(dr, bool)
    idx = [np.arange(f, f + s) % d for f, s, d in zip(fr, sr, dr)]
    inside[np.ix_(*idx)] = True
    assert np.array_equal(out.reshape(dr)[~inside], vr.reshape(dr)[~inside]), case


@pytest.mark.parametrize("seed", range(48))
def test_fuzz_copy(gpu, seed):
    import torch
    import superbblas_amd as sb
    rng = np.random.default_rng(5000 + seed)
    nd = int(rng.integers(1, 7))
    labels = "".join(rng.permutation(list(_LETTERS))[:nd])
    ext = {c: int(rng.integers(1, 6)) for c in labels}
    o0 = labels
    o1 = "".join(rng.permutation(list(labels)))
    d0 = [ext[c] for c in o0]
    d1 = [ext[c] for c in o1]
    f0, s0 = _box(rng, d0)
    f1 = [int(rng.integers(0, d)) for d in d1]
    t0, t1 = [(np.complex128, np.complex128), (np.complex64, np.complex128),
              (np.float64, np.float64), (np.float32, np.complex64),
              (np.int32, np.int32)][int(rng.integers(0, 5))]
    add = bool(rng.integers(0, 2)) and np.dtype(t1).kind != "i"
    alpha = 1.0 if np.dtype(t0).kind == "i" else [1.0, 2.0, -0.5][int(rng.integers(0, 3))]
    v0 = int_valued(_vol(d0), t0, seed) if np.dtype(t0).kind != "i" else \
        np.arange(_vol(d0), dtype=t0)
    v1 = int_valued(_vol(d1), t1, seed + 1) if np.dtype(t1).kind != "i" else \
        -np.arange(_vol(d1), dtype=t1)
    ref = v1.copy()
    oracle_copy(alpha, o0, f0, s0, d0, v0, o1, f1, d1, ref, add=add)
    p0, c0 = _split(sb, gpu, v0, o0, d0, rng)
    p1, c1 = _split(sb, gpu, v1, o1, d1, rng)
    sb.copy(alpha, p0, o0, f0, s0, d0, c0, p1, o1, f1, d1, c1,
            copyadd=sb.Add if add else sb.Copy)
    torch.cuda.synchronize()
    out = _gather(p1, c1, d1, t1)
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8)), (o0, o1, d0, f0, s0, f1, t0,
                                                                     t1, add, alpha)


@pytest.mark.parametrize("seed", range(32))
def test_fuzz_bsr(gpu, seed):
    """bsr_krylov on random stencils: lattice extents 1-4, spin x color blocks (1-4 x 1-3),
    ragged or constant neighbour counts, either block order, row- or column-major x and y,
    alpha/beta; integer-valued data, exact against the oracle's builtin loop."""
    import torch
    import superbblas_amd as sb
    from _common import T_CDOUBLE, oracle_bsr
    rng = np.random.default_rng(9000 + seed)
    L = [int(rng.integers(1, 5)) for _ in range(4)]
    spin, color = int(rng.choice([1, 2, 4])), int(rng.integers(1, 4))
    b = spin * color
    V = _vol(L)
    dim = L + [spin, color]
    sites = np.array(np.unravel_index(np.arange(V), L)).T
    dirs = [(None, 0)] + [(d, s) for d in range(4) for s in (-1, 1)]
    ragged = rng.random() < 0.5
    jj, ii = [], []
    for st in sites:
        k = int(rng.integers(0, 10)) if ragged else 9
        for d, sg in dirs[:k]:
            c = st.copy()
            if d is not None:
                c[d] = (c[d] + sg) % L[d]
            jj.append(list(c) + [0, 0])
        ii.append(k)
    ii = np.array(ii, np.int32)
    jj = np.array(jj, np.int32).reshape(-1, 6) if jj else np.zeros((0, 6), np.int32)
    nnz = int(ii.sum())
    vals = int_valued(nnz * b * b, np.complex128, seed)
    bif = bool(rng.integers(0, 2))
    ncols = int(rng.integers(1, 18))
    x = int_valued(V * b * ncols, np.complex128, seed + 1)
    y0 = int_valued(V * b * ncols, np.complex128, seed + 2)
    xrow, yrow = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
    alpha = [1.0, 2.0, -1.0 + 1.0j][int(rng.integers(0, 3))]
    beta = [0.0, 1.0, 0.5][int(rng.integers(0, 3))]
    ax = np.zeros(V * b * ncols, np.complex128)
    oracle_bsr(T_CDOUBLE, dim, 0, V, b, b, ii, jj.ravel(), vals, bif, x,
               ncols if xrow else V * b, xrow, ax, ncols if yrow else V * b, yrow, ncols, 1.0)
    ref = alpha * ax + beta * y0
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, spin, color]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, bif, [torch.from_numpy(ii).to(gpu)],
                       [torch.from_numpy(jj.ravel().copy()).to(gpu)],
                       [torch.from_numpy(vals).to(gpu)])
    ox = "pXYZTSCn" if xrow else "pnXYZTSC"
    dx = [1] + L + [spin, color, ncols] if xrow else [1, ncols] + L + [spin, color]
    oy = "pxyztscn" if yrow else "pnxyztsc"
    dy = [1] + L + [spin, color, ncols] if yrow else [1, ncols] + L + [spin, color]
    ty = torch.from_numpy(y0.copy()).to(gpu)
    sb.bsr_krylov(alpha, op, "xyztsc", "XYZTSC", [([0] * 8, dx)], ox, [0] * 8, dx, dx,
                  [torch.from_numpy(x).to(gpu)], beta, [([0] * 8, dy)], oy, [0] * 8, dy, dy, "p",
                  [ty])
    torch.cuda.synchronize()
    op.destroy()
    assert np.array_equal(ty.cpu().numpy(), ref), (L, spin, color, ragged, bif, ncols, xrow, yrow,
                                                   alpha, beta)


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_oversize_paths(gpu, seed):
    """The paths for operands beyond 32-bit indexing (copies cut into slabs of the outermost
    destination dimension, GEMMs cut along K / M / N with beta = 1 accumulation), exercised by
    lowering their thresholds (sbx_tune_set copy.max_elems / gemm.max_bytes) on small cases."""
    import superbblas_amd as sb
    sb.tune_set("copy.max_elems", 37)
    sb.tune_set("gemm.max_bytes", 3000)
    try:
        test_fuzz_copy(gpu, seed)
        _fuzz_contraction(gpu, 200 + seed, np.complex128, 1e-10)
    finally:
        sb.tune_set("copy.max_elems", 0)
        sb.tune_set("gemm.max_bytes", 0)


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_bsr_wide(gpu, seed):
    """bsr_krylov across rhs column counts 1-1100 (log-uniform) and every element type, so each
    kernel form's column limits are crossed (the 3x3 row / split / row-chunk kernels, the 12x12
    MFMA kernels, the generic ELL and CSR kernels); 9-point or ragged stencils, integer-valued
    data, exact against the oracle's builtin loop."""
    import torch
    import superbblas_amd as sb
    from _common import NP, T_CDOUBLE, T_CFLOAT, T_DOUBLE, T_FLOAT, oracle_bsr
    rng = np.random.default_rng(7000 + seed)
    t = [T_CDOUBLE, T_CFLOAT, T_DOUBLE, T_FLOAT][seed % 4]
    dt = NP[t]
    L = [int(rng.integers(1, 4)) for _ in range(4)]
    spin, color = [(1, 3), (4, 3), (1, 1), (2, 3)][int(rng.integers(0, 4))]
    b = spin * color
    V = _vol(L)
    dim = L + [spin, color]
    sites = np.array(np.unravel_index(np.arange(V), L)).T
    dirs = [(None, 0)] + [(d, s) for d in range(4) for s in (-1, 1)]
    ragged = rng.random() < 0.25
    jj, ii = [], []
    for st in sites:
        k = int(rng.integers(0, 10)) if ragged else 9
        for d, sg in dirs[:k]:
            c = st.copy()
            if d is not None:
                c[d] = (c[d] + sg) % L[d]
            jj.append(list(c) + [0, 0])
        ii.append(k)
    ii = np.array(ii, np.int32)
    jj = np.array(jj, np.int32).reshape(-1, 6) if jj else np.zeros((0, 6), np.int32)
    nnz = int(ii.sum())
    vals = int_valued(nnz * b * b, dt, seed)
    ncols = int(np.exp(rng.uniform(0, np.log(1100))))
    x = int_valued(V * b * ncols, dt, seed + 1)
    xrow, yrow = bool(rng.random() < 0.75), bool(rng.random() < 0.75)
    ref = np.zeros(V * b * ncols, dt)
    oracle_bsr(t, dim, 0, V, b, b, ii, jj.ravel(), vals, False, x, ncols if xrow else V * b, xrow,
               ref, ncols if yrow else V * b, yrow, ncols, 1.0)
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, spin, color]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, False, [torch.from_numpy(ii).to(gpu)],
                       [torch.from_numpy(jj.ravel().copy()).to(gpu)],
                       [torch.from_numpy(vals).to(gpu)])
    ox = "pXYZTSCn" if xrow else "pnXYZTSC"
    dx = [1] + L + [spin, color, ncols] if xrow else [1, ncols] + L + [spin, color]
    oy = "pxyztscn" if yrow else "pnxyztsc"
    dy = [1] + L + [spin, color, ncols] if yrow else [1, ncols] + L + [spin, color]
    ty = torch.zeros(V * b * ncols, dtype=torch.from_numpy(ref[:1]).dtype, device=gpu)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dx)], ox, [0] * 8, dx, dx,
                  [torch.from_numpy(x).to(gpu)], 0.0, [([0] * 8, dy)], oy, [0] * 8, dy, dy, "p",
                  [ty])
    torch.cuda.synchronize()
    op.destroy()
    assert np.array_equal(ty.cpu().numpy(), ref), (t, L, spin, color, ragged, ncols, xrow, yrow,
                                                   sb.tune_get("bsr.last_kernel"))


@pytest.mark.parametrize("seed", range(40))
def test_fuzz_copy_transpose(gpu, seed):
    """Larger permutations (3-6 labels, extents up to 48, up to ~1M elements, mostly whole boxes)
    so the transpose kernels' planners take part (site-block transpose, block transpose, the tile
    kernel and their paired 8-byte forms); every type pair, Copy / Add, alpha; bit-exact against
    the oracle, and identical with both transpose kernels switched off."""
    import torch
    import superbblas_amd as sb
    rng = np.random.default_rng(6000 + seed)
    nd = int(rng.integers(3, 7))
    labels = "".join(rng.permutation(list(_LETTERS))[:nd])
    while True:
        ext = {c: int(rng.choice([1, 2, 3, 4, 5, 8, 12, 16, 24, 33, 48])) for c in labels}
        if 2000 <= _vol(ext.values()) <= 1 << 20:
            break
    o0 = labels
    o1 = "".join(rng.permutation(list(labels)))
    d0 = [ext[c] for c in o0]
    d1 = [ext[c] for c in o1]
    if rng.random() < 0.8:
        f0, s0 = [0] * nd, list(d0)
    else:
        f0, s0 = _box(rng, d0)
    f1 = [0] * nd if rng.random() < 0.8 else [int(rng.integers(0, d)) for d in d1]
    t0, t1 = [(np.complex128, np.complex128), (np.complex64, np.complex64),
              (np.complex64, np.complex128), (np.complex128, np.complex64),
              (np.float64, np.float64), (np.float32, np.float32), (np.float64, np.complex128),
              (np.int32, np.int32)][seed % 8]
    add = bool(rng.random() < 0.3) and np.dtype(t1).kind != "i"
    alpha = 1.0 if np.dtype(t0).kind == "i" else [1.0, 1.0, -0.5][int(rng.integers(0, 3))]
    v0 = int_valued(_vol(d0), t0, seed) if np.dtype(t0).kind != "i" else \
        np.arange(_vol(d0), dtype=t0)
    v1 = int_valued(_vol(d1), t1, seed + 1) if np.dtype(t1).kind != "i" else \
        -np.arange(_vol(d1), dtype=t1)
    ref = v1.copy()
    oracle_copy(alpha, o0, f0, s0, d0, v0, o1, f1, d1, ref, add=add)
    outs, kinds = [], []
    for off in (0, -1):
        sb.tune_set("copy.trans", off)
        sb.tune_set("copy.btrans", off)
        try:
            t_in = torch.from_numpy(v0).to(gpu)
            t_out = torch.from_numpy(v1.copy()).to(gpu)
            sb.copy(alpha, [([0] * nd, d0)], o0, f0, s0, d0, [t_in], [([0] * nd, d1)], o1, f1, d1,
                    [t_out], copyadd=sb.Add if add else sb.Copy)
            torch.cuda.synchronize()
            kinds.append(sb.tune_get("copy.last_pair"))
        finally:
            sb.tune_set("copy.trans", 0)
            sb.tune_set("copy.btrans", 0)
        outs.append(t_out.cpu().numpy())
    case = (o0, o1, d0, f0, s0, f1, t0, t1, add, alpha, kinds)
    assert np.array_equal(outs[0].view(np.uint8), ref.view(np.uint8)), case
    assert np.array_equal(outs[1].view(np.uint8), ref.view(np.uint8)), case
    assert not kinds[1] & 12, case


@pytest.mark.parametrize("seed", range(96))
def test_fuzz_contraction_large(gpu, seed):
    """Contractions large enough for the matrix-core GEMM forms (LDS-DMA tiles, 48x48 tiles,
    split-K, the shared-operand image, stride forms): T / A / B / C groups of 0-2 labels with
    extents up to 96 and operands up to ~1M elements, whole boxes, random label orders,
    conjugation, alpha / beta, every type; against the oracle within the type's bar."""
    import torch
    import superbblas_amd as sb
    rng = np.random.default_rng(8000 + seed)
    dtype, tol = [(np.complex128, 1e-10), (np.complex64, 2e-5), (np.float64, 1e-12),
                  (np.float32, 2e-5)][seed % 4]
    while True:
        counts = [int(rng.integers(0, 3)) for _ in range(4)]
        counts[1] = max(counts[1], 1)
        if counts[2] + counts[3] == 0:
            counts[2] = 1
        letters = list(rng.permutation(list(_LETTERS)))
        T = "".join(letters[:counts[0]])
        A = "".join(letters[counts[0]:sum(counts[:2])])
        B = "".join(letters[sum(counts[:2]):sum(counts[:3])])
        C = "".join(letters[sum(counts[:3]):sum(counts)])
        ext = {c: int(rng.choice([1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96])) for c in
               T + A + B + C}
        vt, va, vb, vc = (_vol([ext[c] for c in g]) for g in (T, A, B, C))
        if max(vt * va * vb, vt * va * vc, vt * vb * vc) <= 1 << 20 and vt * va * vb * vc <= 4 << 20 \
                and vt * va * vb * vc >= 1 << 14:
            break
    o0 = "".join(rng.permutation(list(T + A + B)))
    o1 = "".join(rng.permutation(list(T + A + C)))
    o_r = "".join(rng.permutation(list(T + B + C)))
    d0, d1, dr = ([ext[c] for c in o] for o in (o0, o1, o_r))
    conj0, conj1 = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
    cplx = np.dtype(dtype).kind == "c"
    alpha = complex(rng.uniform(-2, 2), rng.uniform(-2, 2)) if cplx else float(rng.uniform(-2, 2))
    beta = [0.0, 1.0, 0.5][int(rng.integers(0, 3))]
    v0 = random_valued(_vol(d0), dtype, 3 * seed + 1)
    v1 = random_valued(_vol(d1), dtype, 3 * seed + 2)
    vr = random_valued(_vol(dr), dtype, 3 * seed + 3)
    ref = vr.copy()
    z = lambda d: [0] * len(d)  # noqa: E731
    oracle_contraction(alpha, o0, z(d0), d0, d0, conj0, v0, o1, z(d1), d1, d1, conj1, v1, beta,
                       o_r, z(dr), dr, dr, ref)
    t0, t1, tr = (torch.from_numpy(v.copy()).to(gpu) for v in (v0, v1, vr))
    sb.contraction(alpha, [(z(d0), d0)], z(d0), d0, d0, o0, conj0, [t0], [(z(d1), d1)], z(d1), d1,
                   d1, o1, conj1, [t1], beta, [(z(dr), dr)], z(dr), dr, dr, o_r, [tr])
    torch.cuda.synchronize()
    err = rel_err(tr.cpu().numpy(), ref)
    assert err < tol, (o0, o1, o_r, d0, d1, dr, conj0, conj1, alpha, beta, err)


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_bsr_image_side(gpu, seed):
    """y = alpha A^H x + beta y (x with the image labels; the conjugate-transposed operator built on
    first use) across lattice shapes, block shapes, ragged stencils, block order, 1-600 rhs columns
    and every type; integer-valued data, exact against the oracle's adjoint loop."""
    import torch
    import superbblas_amd as sb
    from _common import NP, T_CDOUBLE, T_CFLOAT, T_DOUBLE, T_FLOAT, oracle_bsr_adjoint
    rng = np.random.default_rng(7500 + seed)
    t = [T_CDOUBLE, T_CFLOAT, T_DOUBLE, T_FLOAT][seed % 4]
    dt = NP[t]
    L = [int(rng.integers(1, 4)) for _ in range(4)]
    spin, color = [(1, 3), (4, 3), (1, 1), (2, 3)][int(rng.integers(0, 4))]
    b = spin * color
    V = _vol(L)
    dim = L + [spin, color]
    sites = np.array(np.unravel_index(np.arange(V), L)).T
    dirs = [(None, 0)] + [(d, s) for d in range(4) for s in (-1, 1)]
    ragged = rng.random() < 0.3
    jj, ii = [], []
    for st in sites:
        k = int(rng.integers(0, 10)) if ragged else 9
        for d, sg in dirs[:k]:
            c = st.copy()
            if d is not None:
                c[d] = (c[d] + sg) % L[d]
            jj.append(list(c) + [0, 0])
        ii.append(k)
    ii = np.array(ii, np.int32)
    jj = np.array(jj, np.int32).reshape(-1, 6) if jj else np.zeros((0, 6), np.int32)
    nnz = int(ii.sum())
    bif = bool(rng.integers(0, 2))
    vals = int_valued(nnz * b * b, dt, seed)
    ncols = int(np.exp(rng.uniform(0, np.log(600))))
    n = V * b * ncols
    x = int_valued(n, dt, seed + 1)
    y0 = int_valued(n, dt, seed + 2)
    beta = [0.0, 1.0][int(rng.integers(0, 2))]
    ax = np.zeros(n, dt)
    oracle_bsr_adjoint(t, dim, 0, V, b, b, ii, jj.ravel(), vals, bif, x, ncols, True, ax, ncols,
                       True, V * b, ncols, 1.0)
    ref = ax + beta * y0
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, spin, color]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, bif, [torch.from_numpy(ii).to(gpu)],
                       [torch.from_numpy(jj.ravel().copy()).to(gpu)],
                       [torch.from_numpy(vals).to(gpu)])
    dx = [1] + L + [spin, color, ncols]
    tx = torch.from_numpy(x).to(gpu)
    ty = torch.from_numpy(y0.copy()).to(gpu)
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", [([0] * 8, dx)], "pxyztscn", [0] * 8, dx, dx, [tx],
                  beta, [([0] * 8, dx)], "pXYZTSCn", [0] * 8, dx, dx, None, [ty])
    torch.cuda.synchronize()
    op.destroy()
    assert np.array_equal(ty.cpu().numpy(), ref.astype(dt)), (t, L, spin, color, ragged, bif,
                                                            ncols, beta)


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_copy_masked(gpu, seed):
    """Masked copies (sbx_copy_masked; the reference's masked local_copy, tensor.h:1019-1027):
    one logical mask over the labels, given to both sides in each side's layout and split with
    each side's components, random permutations, sub-boxes from the origin, Copy / Add, types;
    bit-exact against the oracle's masked copy."""
    import torch
    import superbblas_amd as sb
    from _common import oracle_copy as oc
    rng = np.random.default_rng(5600 + seed)
    nd = int(rng.integers(1, 6))
    labels = "".join(rng.permutation(list(_LETTERS))[:nd])
    while True:
        ext = {c: int(rng.choice([1, 2, 3, 5, 8, 12, 17, 32])) for c in labels}
        if _vol(ext.values()) <= 1 << 18:
            break
    o0 = labels
    o1 = "".join(rng.permutation(list(labels)))
    d0 = [ext[c] for c in o0]
    d1 = [ext[c] for c in o1]
    s0 = [int(rng.integers(1, d + 1)) if rng.random() < 0.4 else d for d in d0]
    t0, t1 = [(np.complex128, np.complex128), (np.complex64, np.complex128), (np.float64, np.float64),
              (np.float32, np.complex64)][seed % 4]
    add = bool(rng.integers(0, 2))
    v0 = int_valued(_vol(d0), t0, seed)
    v1 = int_valued(_vol(d1), t1, seed + 1)
    # the logical mask: a function of the label coordinates, laid out for each side
    salt = {c: int(rng.integers(1, 7)) for c in labels}
    grid0 = np.indices(d0).reshape(nd, -1)
    m0 = (sum(salt[c] * grid0[i] for i, c in enumerate(o0)) % 3 != 0).astype(np.float32)
    grid1 = np.indices(d1).reshape(nd, -1)
    m1 = (sum(salt[c] * grid1[j] for j, c in enumerate(o1)) % 3 != 0).astype(np.float32)
    ref = v1.copy()
    oc(1.0, o0, [0] * nd, s0, d0, v0, o1, [0] * nd, d1, ref, add=add, mask0=m0, mask1=m1)

    def pieces(v, labels_, dims, p):
        full = v.reshape(dims)
        out = []
        for frm, size in p:
            sl = tuple(slice(f, f + s) for f, s in zip(frm, size))
            out.append(torch.from_numpy(np.ascontiguousarray(full[sl]).ravel()).to(gpu))
        return out

    def part(labels_, dims):
        cand = [i for i, d in enumerate(dims) if d >= 2]
        if not cand or rng.random() < 0.5:
            return [([0] * len(dims), list(dims))]
        i = int(rng.choice(cand))
        procs = [1] * len(dims)
        procs[i] = 2
        return sb.basic_partitioning(labels_, dims, procs, labels_[i], 2, 1)

    p0, p1 = part(o0, d0), part(o1, d1)
    c0, c1 = pieces(v0, o0, d0, p0), pieces(v1, o1, d1, p1)
    k0, k1 = pieces(m0, o0, d0, p0), pieces(m1, o1, d1, p1)
    sb.copy(1.0, p0, o0, [0] * nd, s0, d0, c0, p1, o1, [0] * nd, d1, c1,
            copyadd=sb.Add if add else sb.Copy, mask0=k0, mask1=k1)
    torch.cuda.synchronize()
    out = _gather(p1, c1, d1, t1)
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8)), (o0, o1, d0, s0, t0, t1, add)
