"""Pin the oracle (oracle/oracle.c, the CPU restatement) and the library's host planner against
golden vectors produced by the real reference (tests/golden, oracle/ref_golden.cpp).  CPU only."""
import numpy as np
import pytest

from _common import oracle_bsr, oracle_contraction, oracle_copy, oracle_kron_bsr, T_CDOUBLE
from _golden import (CONTRACTION_RTOL, NPT, component_errors, contraction_inputs, gen, manifest,
                     output, parity_masks, vol)


def _is_replicated(p, dim):
    return len(p) > 1 and all(list(s) == list(dim) and not any(f) for f, s in p)


@pytest.mark.parametrize("case", manifest("copy"), ids=lambda c: "copy%d" % c["id"])
def test_oracle_copy(case):
    t0, t1 = NPT[case["t0"]], NPT[case["t1"]]
    v0 = gen(case["gen0"], vol(case["dim0"]), 1, t0)
    v1 = gen(case["gen1"], vol(case["dim1"]), 2, t1)
    reps = len(case["p0"]) if (case["add"] and _is_replicated(case["p0"], case["dim0"])) else 1
    m0, m1 = parity_masks(case) if case.get("mask") else (None, None)
    for _ in range(reps):
        oracle_copy(complex(*case["alpha"]), case["o0"], case["from0"], case["size0"],
                    case["dim0"], v0, case["o1"], case["from1"], case["dim1"], v1,
                    add=case["add"], mask0=m0, mask1=m1)
    ref = output(case, t1)
    assert np.array_equal(v1.view(np.uint8), ref.view(np.uint8))


@pytest.mark.parametrize("case", manifest("contraction"), ids=lambda c: "contr%d" % c["id"])
def test_oracle_contraction(case):
    t = NPT[case["t"]]
    v0, v1, vr = contraction_inputs(case)
    oracle_contraction(complex(*case["alpha"]), case["o0"], case["from0"], case["size0"],
                       case["dim0"], case["conj0"], v0, case["o1"], case["from1"], case["size1"],
                       case["dim1"], case["conj1"], v1, complex(*case["beta"]), case["o_r"],
                       case["fromr"], case["sizer"], case["dimr"], vr)
    ref = output(case, t)
    if case.get("gen", "int") == "int":
        # integer-valued inputs: the sums are exact in f64, so the restatement must match exactly
        assert np.array_equal(vr, ref)
    else:
        # random values: the restatement sums in another order than OpenBLAS
        tol = CONTRACTION_RTOL[case["t"]]
        assert max(component_errors(vr, ref)) < tol


def lattice_operator(L, spin, color):
    """The operator of oracle/ref_golden.cpp bsr_case on one component (whole domain)."""
    b = spin * color
    V = L ** 4
    sites = np.array(np.unravel_index(np.arange(V), (L, L, L, L))).T
    jj = np.zeros((V, 9, 6), np.int32)
    jj[:, 0, :4] = sites
    k = 1
    for d in range(4):
        for s in (-1, 1):
            c = sites.copy()
            c[:, d] = (c[:, d] + s) % L
            jj[:, k, :4] = c
            k += 1
    ii = np.full(V, 9, np.int32)
    vals = gen("int", V * 9 * b * b, 4, np.complex128)
    return ii, jj.reshape(-1), vals


@pytest.mark.parametrize("case", manifest("bsr"), ids=lambda c: "bsr%d" % c["id"])
def test_oracle_bsr(case):
    L, spin, color, ncols = case["L"], case["spin"], case["color"], case["ncols"]
    power = case.get("power", 1)
    b = spin * color
    V = L ** 4
    ii, jj, vals = lattice_operator(L, spin, color)
    # powers (bsr.h:2211-2247): y[p] = A^(p+1) x
    cur, out = gen("int", V * b * ncols, 5, np.complex128), []
    for _ in range(power):
        y = np.zeros_like(cur)
        oracle_bsr(T_CDOUBLE, [L, L, L, L, spin, color], 0, V, b, b, ii, jj, vals, False, cur,
                   ncols, True, y, ncols, True, ncols, 1.0)
        out.append(y)
        cur = y
    assert np.array_equal(np.concatenate(out), output(case, np.complex128))


@pytest.mark.parametrize("case", manifest("kron_bsr"), ids=lambda c: "kron%d" % c["id"])
def test_oracle_kron_bsr(case):
    """Kronecker BSR (create_lattice_kron, tests/bsr.cpp:547-644) against the reference."""
    L, spin, color, ncols = case["L"], case["spin"], case["color"], case["ncols"]
    V = L ** 4
    ii, jj, _ = lattice_operator(L, 1, 1)
    vals = gen("int", V * 9 * color * color, 4, np.complex128)
    kron = gen("int", 9 * spin * spin, 7, np.complex128)
    cur, out = gen("int", V * color * ncols * spin, 5, np.complex128), []
    for _ in range(case["power"]):
        y = np.zeros_like(cur)
        oracle_kron_bsr(T_CDOUBLE, [L, L, L, L, 1, 1], 0, V, 9, color, color, spin, spin, jj,
                        vals, kron, case["block_im_fast"], cur, y, ncols, 1.0)
        out.append(y)
        cur = y
    assert np.array_equal(np.concatenate(out), output(case, np.complex128))


# ---- host planner (the library's C++ partitioning helpers; no GPU needed) ----

def test_partitioning_distributed_procs():
    import superbblas_amd as sb
    for c in manifest("pdp"):
        assert sb.partitioning_distributed_procs(c["order"], c["dim"], c["dist"],
                                                 c["nprocs"]) == c["procs"], c


def test_basic_partitioning():
    import superbblas_amd as sb
    for c in manifest("bp"):
        p = sb.basic_partitioning(c["order"], c["dim"], c["procs"], c["dist"], c["nprocs"],
                                  c["ncomponents"])
        assert [[list(f), list(s)] for f, s in p] == c["p"], c


def test_basic_partitioning_ext():
    import superbblas_amd as sb
    for c in manifest("bpe"):
        p = sb.basic_partitioning_ext(c["dim"], c["procs"], c["nprocs"], c["replicate"], c["ext"])
        assert [[list(f), list(s)] for f, s in p] == c["p"], c


def test_make_hole():
    import superbblas_amd as sb
    for c in manifest("hole"):
        r = sb.make_hole(c["from"], c["size"], c["hfrom"], c["hsize"], c["dim"])
        assert [[list(f), list(s)] for f, s in r] == c["r"], c


def test_oracle_bsr_adjoint_identity():
    """The A^H restatement (the reference's CPU path has none: bsr.h:536-538) is pinned through
    the golden-pinned forward product: <y, A x> = <A^H y, x> on the lattice operator."""
    from _common import oracle_bsr_adjoint
    L, spin, color, ncols = 4, 1, 3, 2
    b = spin * color
    V = L ** 4
    ii, jj, vals = lattice_operator(L, spin, color)
    x = gen("int", V * b * ncols, 5, np.complex128)
    y = gen("int", V * b * ncols, 6, np.complex128)
    ax = np.zeros_like(x)
    oracle_bsr(T_CDOUBLE, [L, L, L, L, spin, color], 0, V, b, b, ii, jj, vals, False, x, ncols,
               True, ax, ncols, True, ncols, 1.0)
    ahy = np.zeros_like(y)
    oracle_bsr_adjoint(T_CDOUBLE, [L, L, L, L, spin, color], 0, V, b, b, ii, jj, vals, False, y,
                       ncols, True, ahy, ncols, True, V * b, ncols, 1.0)
    assert np.vdot(y, ax) == np.vdot(ahy, x)


# ---- dense batched solvers (dense.h) ----

def _cm(m):
    """(nb, n, n) [b, r, c] -> column-major data per matrix"""
    return np.ascontiguousarray(m.transpose(0, 2, 1)).ravel()


def _from_cm(d, nb, r, c):
    return d.reshape(nb, c, r).transpose(0, 2, 1)


def _dense_tol(t):
    return 1e-12 if np.dtype(t) in (np.float64, np.complex128) else 1e-5


@pytest.mark.parametrize("case", manifest("cholesky") + manifest("inversion"),
                         ids=lambda c: "%s%d" % (c["kind"], c["id"]))
def test_oracle_dense_inplace(case):
    from _common import oracle_getrf, oracle_getrs, oracle_potrf
    from _dense import dense_input, from_matrices, to_matrices
    t = NPT[case["t"]]
    o, dim, n = case["o"], case["dim"], case["n"]
    nt = dim[0]
    a = dense_input(case["input"], nt, n, t)  # [t, r, c]
    # lay the input out as the tensor o (t + rows + cols), as the golden generator did
    g = from_matrices(a, "t" + case["orows"] + case["ocols"],
                      [dim[o.index(c)] for c in "t" + case["orows"] + case["ocols"]],
                      case["orows"], case["ocols"])
    g = to_matrices(g, "t" + case["orows"] + case["ocols"],
                    [dim[o.index(c)] for c in "t" + case["orows"] + case["ocols"]],
                    case["orows"], case["ocols"])
    w = _cm(g).astype(t)
    if case["kind"] == "cholesky":
        assert oracle_potrf(w, n, nt) == 0
    else:
        piv = np.zeros(nt * n, np.int32)
        assert oracle_getrf(w, n, nt, piv) == 0
        eye = np.tile(np.eye(n, dtype=t).ravel(), nt)
        assert oracle_getrs(w, n, nt, piv, n, eye) == 0
        w = eye
    res = _from_cm(w, nt, n, n)
    ref = to_matrices(output(case, t), o, dim, case["orows"], case["ocols"])
    assert np.allclose(res, ref, rtol=0, atol=_dense_tol(t) * np.abs(ref).max())


@pytest.mark.parametrize("case", manifest("trsm") + manifest("gesm"),
                         ids=lambda c: "%s%d" % (c["kind"], c["id"]))
def test_oracle_dense_solve(case):
    from _common import oracle_getrf, oracle_getrs, oracle_trsm
    from _dense import dense_input, from_panel, to_panel
    t = NPT[case["t"]]
    oc, n = case["oc"], case["n"]
    nt = case["dimc"][0]
    c = dense_input("tri" if case["kind"] == "trsm" else "gen", nt, n, t)
    ox, oy, dimx, dimy = case["ox"], case["oy"], case["dimx"], case["dimy"]
    x = gen("int", vol(dimx), 5, t)
    alpha = complex(*case["alpha"]) if np.dtype(t).kind == "c" else case["alpha"][0]
    rows, cols = case["orows"], case["ocols"]
    on = [l for l in ox if l not in oc]
    contract_rows = any(l in rows for l in ox)
    cw = _cm(c)
    if not contract_rows:  # C \\ X: X (n x m), rows = column labels
        xm = to_panel(x, ox, dimx, on, cols)  # [b, m, n] = column-major (n x m)
        m = xm.shape[1]
        xw = np.ascontiguousarray(xm).ravel().astype(t)
        if case["kind"] == "trsm":
            oracle_trsm(True, n, nt, m, alpha, cw, xw)
        else:
            piv = np.zeros(nt * n, np.int32)
            assert oracle_getrf(cw, n, nt, piv) == 0
            oracle_getrs(cw, n, nt, piv, m, xw)
            xw = xw * alpha
        res = from_panel(xw.reshape(nt, m, n), oy, dimy, on, rows)
    else:  # X / C: X (m x n), columns = row labels
        xm = to_panel(x, ox, dimx, rows, on)  # [b, n, m] = column-major (m x n)
        m = xm.shape[2]
        xw = np.ascontiguousarray(xm).ravel().astype(t)
        oracle_trsm(False, n, nt, m, alpha, cw, xw)
        res = from_panel(xw.reshape(nt, n, m), oy, dimy, cols, on)
    ref = output(case, t)
    assert np.allclose(res, ref, rtol=0, atol=_dense_tol(t) * np.abs(ref).max())
