"""Shared test helpers: the oracle (CPU restatement, oracle/oracle.c) through ctypes, and
deterministic test data.  Test infrastructure only."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")

T_FLOAT, T_DOUBLE, T_CFLOAT, T_CDOUBLE, T_INT, T_SIZE_T = range(6)
NP = {T_FLOAT: np.float32, T_DOUBLE: np.float64, T_CFLOAT: np.complex64,
      T_CDOUBLE: np.complex128, T_INT: np.int32, T_SIZE_T: np.uint64}
TYPE_OF = {np.dtype(v): k for k, v in NP.items()}

_oracle = None


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"])
        _oracle = ctypes.CDLL(ORACLE_SO)
    return _oracle


def ints(xs):
    return (ctypes.c_int * max(1, len(xs)))(*[int(x) for x in xs])


def scal(a):
    a = complex(a)
    return (ctypes.c_double * 2)(a.real, a.imag)


def ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def oracle_copy(alpha, o0, from0, size0, dim0, v0, o1, from1, dim1, v1, co=0, add=False,
                mask0=None, mask1=None):
    """In place on v1 (numpy); optional float32 masks over the whole origin / destination."""
    m0 = ptr(mask0) if mask0 is not None else None
    m1 = ptr(mask1) if mask1 is not None else None
    rc = oracle().oracle_copy_masked(len(o0), len(o1), scal(alpha), TYPE_OF[v0.dtype],
                                     TYPE_OF[v1.dtype], o0.encode(), ints(from0), ints(size0),
                                     ints(dim0), ptr(v0), m0, o1.encode(), ints(from1),
                                     ints(dim1), ptr(v1), m1, co, int(add))
    assert rc == 0, "oracle_copy_masked: %d" % rc


def oracle_contraction(alpha, o0, from0, size0, dim0, conj0, v0, o1, from1, size1, dim1, conj1,
                       v1, beta, o_r, fromr, sizer, dimr, vr, co=0):
    rc = oracle().oracle_contraction(
        TYPE_OF[v0.dtype], len(o0), o0.encode(), ints(from0), ints(size0), ints(dim0), int(conj0),
        ptr(v0), len(o1), o1.encode(), ints(from1), ints(size1), ints(dim1), int(conj1), ptr(v1),
        len(o_r), o_r.encode(), ints(fromr), ints(sizer), ints(dimr), ptr(vr), scal(alpha),
        scal(beta), co)
    assert rc == 0


def oracle_gemm(ta, tb, m, n, k, alpha, a, lda, sa, b, ldb, sb, beta, c, ldc, sc, batch):
    o = oracle()
    o.oracle_xgemm_batch_strided.argtypes = [
        ctypes.c_int, ctypes.c_char, ctypes.c_char, ctypes.c_int, ctypes.c_int, ctypes.c_int,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_void_p,
        ctypes.c_int, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
        ctypes.c_long, ctypes.c_int]
    rc = o.oracle_xgemm_batch_strided(TYPE_OF[c.dtype], ta.encode(), tb.encode(), m, n, k,
                                      ctypes.cast(scal(alpha), ctypes.c_void_p), ptr(a), lda, sa,
                                      ptr(b), ldb, sb, ctypes.cast(scal(beta), ctypes.c_void_p),
                                      ptr(c), ldc, sc, batch)
    assert rc == 0


def oracle_bsr(t, dimd, co, block_rows, bi, bd, ii, jj, v, block_im_fast, x, ldx, x_row_major,
               y, ldy, y_row_major, ncols, alpha, add=False):
    o = oracle()
    o.oracle_bsr.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_int,
        ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
        ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_void_p, ctypes.c_long,
        ctypes.c_int, ctypes.c_long, ctypes.c_void_p, ctypes.c_int]
    rc = o.oracle_bsr(t, len(dimd), ctypes.cast(ints(dimd), ctypes.c_void_p), co, block_rows, bi,
                      bd, ptr(ii), ptr(jj), ptr(v), int(block_im_fast), ptr(x), ldx,
                      int(x_row_major), ptr(y), ldy, int(y_row_major), ncols,
                      ctypes.cast(scal(alpha), ctypes.c_void_p), int(add))
    assert rc == 0


def oracle_bsr_adjoint(t, dimd, co, block_rows, bi, bd, ii, jj, v, block_im_fast, x, ldx,
                       x_row_major, y, ldy, y_row_major, ydim, ncols, alpha, add=False):
    """y = alpha A^H x on one component (x by image rows, y by domain rows)."""
    o = oracle()
    o.oracle_bsr_adjoint.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_int,
        ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
        ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_void_p, ctypes.c_long,
        ctypes.c_int, ctypes.c_long, ctypes.c_long, ctypes.c_void_p, ctypes.c_int]
    rc = o.oracle_bsr_adjoint(t, len(dimd), ctypes.cast(ints(dimd), ctypes.c_void_p), co,
                              block_rows, bi, bd, ptr(ii), ptr(jj), ptr(v), int(block_im_fast),
                              ptr(x), ldx, int(x_row_major), ptr(y), ldy, int(y_row_major), ydim,
                              ncols, ctypes.cast(scal(alpha), ctypes.c_void_p), int(add))
    assert rc == 0


def oracle_kron_bsr(t, site_dim, co, block_rows, nnz, bi, bd, ki, kd, jj, v, kron, block_im_fast,
                    x, y, ncols, alpha, add=False):
    """Kronecker BSR on one component, x (site, d, col, b) and y (row, i, col, a) row major."""
    o = oracle()
    o.oracle_kron_bsr.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_int,
        ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long,
        ctypes.c_void_p, ctypes.c_int]
    rc = o.oracle_kron_bsr(t, len(site_dim), ctypes.cast(ints(site_dim), ctypes.c_void_p), co,
                           block_rows, nnz, bi, bd, ki, kd, ptr(jj), ptr(v), ptr(kron),
                           int(block_im_fast), ptr(x), ptr(y), ncols,
                           ctypes.cast(scal(alpha), ctypes.c_void_p), int(add))
    assert rc == 0


def oracle_potrf(a, n, k):
    return oracle().oracle_potrf_upper(TYPE_OF[a.dtype], ctypes.c_long(n), ctypes.c_long(k), ptr(a))


def oracle_getrf(a, n, k, ipiv):
    return oracle().oracle_getrf(TYPE_OF[a.dtype], ctypes.c_long(n), ctypes.c_long(k), ptr(a),
                                 ptr(ipiv))


def oracle_getrs(a, n, k, ipiv, m, b):
    return oracle().oracle_getrs(TYPE_OF[a.dtype], ctypes.c_long(n), ctypes.c_long(k), ptr(a),
                                 ptr(ipiv), ctypes.c_long(m), ptr(b))


def oracle_trsm(left, n, k, m, alpha, a, x):
    return oracle().oracle_trsm_upper(TYPE_OF[a.dtype], int(left), ctypes.c_long(n),
                                      ctypes.c_long(k), ctypes.c_long(m),
                                      ctypes.cast(scal(alpha), ctypes.c_void_p), ptr(a), ptr(x))


def int_valued(n, dtype, seed=0):
    """Small integer-valued data (exact in every supported type)."""
    i = np.arange(n, dtype=np.int64) + seed * 7919
    re = ((i * 7 + 3) % 11 - 5).astype(np.float64)
    im = ((i * 5 + 1) % 13 - 6).astype(np.float64)
    dt = np.dtype(dtype)
    if dt.kind == "c":
        return (re + 1j * im).astype(dt)
    return re.astype(dt)


def random_valued(n, dtype, seed=0):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if dt.kind == "c":
        return (rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)).astype(dt)
    return rng.uniform(-1, 1, n).astype(dt)


def index_valued(n, dtype):
    """Every element holds its own global index (the reference's mock-index tensors,
    dist.h:1919-2116)."""
    i = np.arange(n, dtype=np.int64)
    dt = np.dtype(dtype)
    if dt.kind == "c":
        out = np.empty(n, dt)
        out.real = i
        out.imag = -i.astype(np.float64)
        return out
    return i.astype(dt)


def rel_err(a, b):
    a = np.asarray(a, dtype=np.complex128).ravel()
    b = np.asarray(b, dtype=np.complex128).ravel()
    den = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (den if den > 0 else 1.0)


def stencil_jj(dims, kind="stencil", rng=None, cut=None):
    """jj coordinates (x y z t s c) of a periodic 9-point stencil on `dims`, or 9 random sites;
    `cut`: blocks whose neighbour crosses dimension 0 past that coordinate get column -1"""
    vol = int(np.prod(dims))
    sites = np.array(np.unravel_index(np.arange(vol), dims)).T
    jj = np.zeros((vol, 9, 6), np.int32)
    if kind == "random":
        jj[:, :, :4] = sites[rng.integers(0, vol, (vol, 9))]
        return jj
    jj[:, 0, :4] = sites
    k = 1
    for d in range(4):
        for s in (-1, 1):
            c = sites.copy()
            c[:, d] = (c[:, d] + s) % dims[d]
            jj[:, k, :4] = c
            if cut is not None and d == 0:
                jj[(sites[:, 0] + s < 0) | (sites[:, 0] + s >= cut), k, 0] = -1
            k += 1
    return jj
