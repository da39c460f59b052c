"""Dense batched solvers on the GPU (dense.h: cholesky / trsm / gesm / inversion) against the
reference's outputs (tests/golden, made by the real reference with LAPACK) and the oracle's
restatement; tolerances relative to the largest entry (1e-12 for double precision, 1e-5 for
single)."""
import numpy as np
import pytest

from _golden import NPT, gen, manifest, output, piece, put_piece, vol

pytestmark = pytest.mark.gpu


def _tol(t):
    return 1e-12 if np.dtype(t) in (np.float64, np.complex128) else 2e-5


def _scatter(glob, dim, p, gpu):
    import torch
    return [torch.from_numpy(piece(glob, dim, f, s)).to(gpu) for f, s in p]


def _gather(comps, dim, p, dtype):
    g = np.zeros(vol(dim), dtype)
    for (f, s), c in zip(p, comps):
        if vol(s):
            put_piece(g, dim, f, s, c.cpu().numpy())
    return g


def _close(a, b, t):
    return np.allclose(a, b, rtol=0, atol=_tol(t) * max(1.0, np.abs(b).max()))


@pytest.mark.parametrize("case", manifest("cholesky") + manifest("inversion"),
                         ids=lambda c: "%s%d" % (c["kind"], c["id"]))
def test_golden_dense_inplace(gpu, case):
    import torch
    import superbblas_amd as sb
    from _dense import dense_input, from_matrices
    t = NPT[case["t"]]
    o, dim, n = case["o"], case["dim"], case["n"]
    a = dense_input(case["input"], dim[0], n, t)
    g = from_matrices(a, o, dim, case["orows"], case["ocols"])
    v = _scatter(g, dim, case["p"], gpu)
    (sb.cholesky if case["kind"] == "cholesky" else sb.inversion)(
        case["p"], dim, o, v, case["orows"], case["ocols"])
    torch.cuda.synchronize()
    out = _gather(v, dim, case["p"], t)
    assert _close(out, output(case, t), t)


@pytest.mark.parametrize("case", manifest("trsm") + manifest("gesm"),
                         ids=lambda c: "%s%d" % (c["kind"], c["id"]))
@pytest.mark.parametrize("wave", [2, 1, 0])
def test_golden_dense_solve(gpu, case, wave):
    """The reference's trsm / gesm outputs, with the small-matrix wave kernels (dense.wave 2:
    the triangular solves too, 1: the LU) and with the workgroup-per-matrix kernels (0)."""
    import torch
    import superbblas_amd as sb
    old = sb.tune_get("dense.wave")
    sb.tune_set("dense.wave", wave)
    try:
        _golden_solve(gpu, case)
    finally:
        sb.tune_set("dense.wave", old)


def _golden_solve(gpu, case):
    import torch
    import superbblas_amd as sb
    from _dense import dense_input, from_matrices
    t = NPT[case["t"]]
    oc, dimc, n = case["oc"], case["dimc"], case["n"]
    c = dense_input("tri" if case["kind"] == "trsm" else "gen", dimc[0], n, t)
    gc = from_matrices(c, oc, dimc, case["orows"], case["ocols"])
    gx = gen("int", vol(case["dimx"]), 5, t)
    gy = gen("int", vol(case["dimy"]), 6, t)
    vc = _scatter(gc, dimc, case["pc"], gpu)
    vx = _scatter(gx, case["dimx"], case["px"], gpu)
    vy = _scatter(gy, case["dimy"], case["py"], gpu)
    alpha = complex(*case["alpha"]) if np.dtype(t).kind == "c" else case["alpha"][0]
    (sb.trsm if case["kind"] == "trsm" else sb.gesm)(
        alpha, case["pc"], dimc, oc, vc, case["orows"], case["ocols"], case["px"], case["dimx"],
        case["ox"], vx, case["py"], case["dimy"], case["oy"], vy)
    torch.cuda.synchronize()
    out = _gather(vy, case["dimy"], case["py"], t)
    assert _close(out, output(case, t), t)


@pytest.mark.parametrize("dtype", [np.complex128, np.float64, np.complex64, np.float32])
@pytest.mark.parametrize("n,wave", [(5, 1), (5, 0), (12, 1), (12, 0), (16, 1), (3, 1), (100, 1)])
def test_dense_types_sizes(gpu, dtype, n, wave):
    """Up to 16 x 16 a wave per matrix (dense.wave 1; 0: the workgroup-per-matrix kernels);
    n = 100 exceeds the LDS staging (global-memory path for complex<double> / double)."""
    import torch
    import superbblas_amd as sb
    from _common import oracle_getrf, oracle_getrs, oracle_potrf
    from _dense import dense_input
    old = sb.tune_get("dense.wave")
    sb.tune_set("dense.wave", wave)
    try:
        _types_sizes(gpu, dtype, n)
    finally:
        sb.tune_set("dense.wave", old)


def _types_sizes(gpu, dtype, n):
    import torch
    import superbblas_amd as sb
    from _common import oracle_getrf, oracle_getrs, oracle_potrf
    from _dense import dense_input
    nt = 6
    full = [([0, 0, 0], [nt, n, n])]
    dim = [nt, n, n]
    # Cholesky of an HPD matrix (tij: the column index fastest in memory)
    a = dense_input("hpd", nt, n, dtype)
    v = [torch.from_numpy(a.ravel().copy()).to(gpu)]
    sb.cholesky(full, dim, "tij", v, "i", "j")
    w = np.ascontiguousarray(a.astype(np.complex128).transpose(0, 2, 1)).ravel()
    assert oracle_potrf(w, n, nt) == 0
    ref = w.reshape(nt, n, n).transpose(0, 2, 1)
    out = v[0].cpu().numpy().reshape(nt, n, n)
    assert _close(out, ref.astype(dtype) if np.dtype(dtype).kind == "c" else ref.real, dtype)
    # inversion of a diagonally dominant matrix
    g = dense_input("gen", nt, n, dtype)
    v = [torch.from_numpy(g.ravel().copy()).to(gpu)]
    sb.inversion(full, dim, "tij", v, "i", "j")
    w = np.ascontiguousarray(g.astype(np.complex128).transpose(0, 2, 1)).ravel()
    piv = np.zeros(nt * n, np.int32)
    assert oracle_getrf(w, n, nt, piv) == 0
    eye = np.tile(np.eye(n, dtype=np.complex128).ravel(), nt)
    oracle_getrs(w, n, nt, piv, n, eye)
    ref = eye.reshape(nt, n, n).transpose(0, 2, 1)
    out = v[0].cpu().numpy().reshape(nt, n, n)
    assert _close(out, ref.astype(dtype) if np.dtype(dtype).kind == "c" else ref.real, dtype)


def test_dense_errors(gpu):
    import torch
    import superbblas_amd as sb
    n, nt = 4, 2
    full = [([0, 0, 0], [nt, n, n])]
    a = -np.eye(n)[None].repeat(nt, 0)  # not positive definite
    v = [torch.from_numpy(a.ravel().copy()).to(gpu)]
    with pytest.raises(sb.SuperbblasError, match="lapack routine: 1"):
        sb.cholesky(full, [nt, n, n], "tij", v, "i", "j")
    z = [torch.zeros(nt * n * n, dtype=torch.float64, device=gpu)]  # singular
    with pytest.raises(sb.SuperbblasError, match="lapack routine: 1"):
        sb.inversion(full, [nt, n, n], "tij", z, "i", "j")
    with pytest.raises(sb.SuperbblasError, match="share labels"):
        sb.cholesky(full, [nt, n, n], "tij", v, "i", "i")
    x = [torch.zeros(nt * n * 2, dtype=torch.float64, device=gpu)]
    px = [([0, 0, 0], [nt, 2, n])]
    with pytest.raises(sb.SuperbblasError, match="row labels"):
        sb.gesm(1.0, full, [nt, n, n], "tij", v, "i", "j", px, [nt, 2, n], "tni", x, px,
                [nt, 2, n], "tnj", x)


@pytest.mark.parametrize("wave", [1, 0])
def test_dense_failure_flag(gpu, wave):
    """a failure late in a large batch is reported with its LAPACK info (the host-mapped failure
    flag, then the search for the first failed matrix), and the next call on the same thread sees a
    clear flag: a good batch after a failed one succeeds"""
    import torch
    import superbblas_amd as sb
    n, nt = 12, 300
    dim = [nt, n, n]
    full = [([0, 0, 0], dim)]
    old = sb.tune_get("dense.wave")
    sb.tune_set("dense.wave", wave)
    try:
        good = np.tile((np.eye(n) * 4 + 0.1).ravel(), nt)
        bad = good.reshape(nt, n, n).copy()
        bad[217, :, 5] = 0  # column 5 of matrix 217: LU stops at pivot 6
        with pytest.raises(sb.SuperbblasError, match="lapack routine: 6"):
            sb.inversion(full, dim, "tij", [torch.from_numpy(bad.ravel().copy()).to(gpu)], "i", "j")
        v = torch.from_numpy(good.copy()).to(gpu)
        sb.inversion(full, dim, "tij", [v], "i", "j")
        ref = np.linalg.inv(good.reshape(nt, n, n))
        assert np.abs(v.cpu().numpy().reshape(nt, n, n) - ref).max() < 1e-12
        hp = np.tile(np.eye(n).ravel() * 2.0, nt).reshape(nt, n, n)
        hp[299, 4, 4] = -1.0  # not positive definite at pivot 5
        with pytest.raises(sb.SuperbblasError, match="lapack routine: 5"):
            sb.cholesky(full, dim, "tij", [torch.from_numpy(hp.ravel().copy()).to(gpu)], "i", "j")
        u = torch.from_numpy(np.tile(np.eye(n).ravel() * 4.0, nt)).to(gpu)
        sb.cholesky(full, dim, "tij", [u], "i", "j")
        assert np.allclose(u.cpu().numpy().reshape(nt, n, n)[:, range(n), range(n)], 2.0)
    finally:
        sb.tune_set("dense.wave", old)
