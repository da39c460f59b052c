"""contraction() on the GPU vs the oracle's label einsum (dist.h:3701-3731 semantics).
Tolerance 1e-10 relative (Frobenius) for complex<double>/double (north_star)."""
import numpy as np
import pytest

from _common import int_valued, oracle_contraction, random_valued, rel_err

pytestmark = pytest.mark.gpu


def _vol(d):
    n = 1
    for x in d:
        n *= x
    return n


def _single(dim):
    return [([0] * len(dim), list(dim))]


def _gpu_contraction(gpu, alpha, o0, from0, size0, dim0, conj0, v0, o1, from1, size1, dim1,
                     conj1, v1, beta, o_r, fromr, sizer, dimr, vr, co=0):
    import torch
    import superbblas_amd as sb
    t0, t1, tr = (torch.from_numpy(x).to(gpu) for x in (v0, v1, vr))
    sb.contraction(alpha, _single(dim0), from0, size0, dim0, o0, conj0, [t0], _single(dim1),
                   from1, size1, dim1, o1, conj1, [t1], beta, _single(dimr), fromr, sizer, dimr,
                   o_r, [tr], co=co)
    torch.cuda.synchronize()
    return tr.cpu().numpy()


def _lattice(L, n, o0, o1, dtype=np.complex128):
    sizes = {"t": L, "x": L, "y": L, "z": L, "s": 4, "c": 3, "n": n, "N": n, "S": 4}
    d0 = [sizes[c] for c in o0]
    d1 = [sizes[c] for c in o1]
    dr = [sizes[c] for c in "tNSns"]
    return d0, d1, dr


@pytest.mark.parametrize("o0,o1", [("tnsxyzc", "tNSxyzc"), ("tsxyzcn", "tSxyzcN")])
def test_lattice_contraction(gpu, o0, o1):
    """dist.cpp:364-415: the column- and row-major lattice contractions (4^4, n = 4)."""
    d0, d1, dr = _lattice(4, 4, o0, o1)
    v0 = random_valued(_vol(d0), np.complex128, 1)
    v1 = random_valued(_vol(d1), np.complex128, 2)
    vr = random_valued(_vol(dr), np.complex128, 3)
    ref = vr.copy()
    z = lambda d: [0] * len(d)
    oracle_contraction(1.0, o0, z(d0), d0, d0, False, v0, o1, z(d1), d1, d1, False, v1, 0.0,
                       "tNSns", z(dr), dr, dr, ref)
    out = _gpu_contraction(gpu, 1.0, o0, z(d0), d0, d0, False, v0, o1, z(d1), d1, d1, False, v1,
                           0.0, "tNSns", z(dr), dr, dr, vr.copy())
    assert rel_err(out, ref) < 1e-10


_T, _A, _B, _C = "ABCD", "IJKL", "QRST", "YZWV"


def _random_case(rng, dtype):
    nT, nA, nB, nC = (int(x) for x in rng.integers(0, 3, 4))
    T, A, B, C = _T[:nT], _A[:nA], _B[:nB], _C[:nC]
    size = {c: int(rng.integers(1, 4)) for c in T + A + B + C}

    def order(s):
        return "".join(rng.permutation(list(s))) if s else ""
    o0, o1, o_r = order(T + A + B), order(T + A + C), order(T + B + C)
    if not o0 or not o1 or not o_r:
        return None
    res = []
    for o in (o0, o1, o_r):
        sz = [size[c] for c in o]
        frm = [int(rng.integers(0, 2)) for _ in o]
        dim = [f + s for f, s in zip(frm, sz)]  # as contract.cpp:160-168
        res.append((o, frm, sz, dim))
    conj0, conj1 = (bool(x) for x in rng.integers(0, 2, 2))
    if np.dtype(dtype).kind != "c":
        conj0 = conj1 = False
    alpha = [1.0, -1.0, 0.5, 1.5 - 0.5j][int(rng.integers(0, 4))]
    beta = [0.0, 1.0, -1.0, 0.25 + 1j][int(rng.integers(0, 4))]
    if np.dtype(dtype).kind != "c":
        alpha, beta = alpha.real if isinstance(alpha, complex) else alpha, \
            beta.real if isinstance(beta, complex) else beta
    return res, conj0, conj1, alpha, beta


@pytest.mark.parametrize("dtype", [np.complex128, np.float64])
def test_random_label_orders(gpu, dtype):
    """contract.cpp-style cases: every T/A/B/C group combination, random label orders, periodic
    boxes (from != 0), conjugation, alpha/beta (contract.cpp:276-338, 341-420)."""
    rng = np.random.default_rng(11)
    done = 0
    while done < 60:
        case = _random_case(rng, dtype)
        if case is None:
            continue
        (t0, t1, tr), conj0, conj1, alpha, beta = case
        v0 = int_valued(_vol(t0[3]), dtype, 1)
        v1 = int_valued(_vol(t1[3]), dtype, 2)
        vr = int_valued(_vol(tr[3]), dtype, 3)
        ref = vr.copy()
        oracle_contraction(alpha, t0[0], t0[1], t0[2], t0[3], conj0, v0, t1[0], t1[1], t1[2],
                           t1[3], conj1, v1, beta, tr[0], tr[1], tr[2], tr[3], ref)
        out = _gpu_contraction(gpu, alpha, t0[0], t0[1], t0[2], t0[3], conj0, v0, t1[0], t1[1],
                               t1[2], t1[3], conj1, v1, beta, tr[0], tr[1], tr[2], tr[3],
                               vr.copy())
        assert rel_err(out, ref) < 1e-10, (case, done)
        done += 1


def test_multicomponent_contraction(gpu):
    """The lattice contraction with operands split in 2 and 3 components over different labels
    (forces redistribution), output on one component."""
    import torch
    import superbblas_amd as sb
    d0, d1, dr = _lattice(4, 2, "tnsxyzc", "tNSxyzc")
    v0 = random_valued(_vol(d0), np.complex128, 1)
    v1 = random_valued(_vol(d1), np.complex128, 2)
    vr = random_valued(_vol(dr), np.complex128, 3)
    ref = vr.copy()
    z = lambda d: [0] * len(d)
    oracle_contraction(1.0, "tnsxyzc", z(d0), d0, d0, False, v0, "tNSxyzc", z(d1), d1, d1, False,
                       v1, 1.0, "tNSns", z(dr), dr, dr, ref)
    p0 = sb.basic_partitioning("tnsxyzc", d0, [1, 1, 1, 2, 1, 1, 1], "x", 2, 1)
    p1 = sb.basic_partitioning("tNSxyzc", d1, [1, 1, 1, 1, 1, 3, 1], "z", 3, 1)

    def split(v, dims, p):
        full = v.reshape(dims)
        out = []
        for frm, size in p:
            sl = tuple(slice(f, f + s) for f, s in zip(frm, size))
            out.append(torch.from_numpy(np.ascontiguousarray(full[sl]).ravel()).to(gpu))
        return out
    c0, c1 = split(v0, d0, p0), split(v1, d1, p1)
    cr = [torch.from_numpy(vr.copy()).to(gpu)]
    sb.contraction(1.0, p0, z(d0), d0, d0, "tnsxyzc", False, c0, p1, z(d1), d1, d1, "tNSxyzc",
                   False, c1, 1.0, _single(dr), z(dr), dr, dr, "tNSns", cr)
    torch.cuda.synchronize()
    assert rel_err(cr[0].cpu().numpy(), ref) < 1e-10


@pytest.mark.parametrize("case", ["tslice", "nslice", "xbox", "twrap", "all_t_in_r"])
def test_subbox_contraction(gpu, case):
    """contraction() on boxes smaller than the tensors (from/size): t slices and n slices run
    in place on views of the components; an x box and a periodic t box that wraps go through
    temporaries.  Elements of vr outside the box stay untouched."""
    L, n = 4, 4
    d0, d1, dr = _lattice(L, n, "tnsxyzc", "tNSxyzc")
    v0 = random_valued(_vol(d0), np.complex128, 11)
    v1 = random_valued(_vol(d1), np.complex128, 12)
    vr = random_valued(_vol(dr), np.complex128, 13)
    f0, s0 = [0] * 7, list(d0)
    f1, s1 = [0] * 7, list(d1)
    fr, sr = [0] * 5, list(dr)
    if case == "tslice":
        f0[0] = f1[0] = fr[0] = 1
        s0[0] = s1[0] = sr[0] = 2
    elif case == "nslice":
        f0[1], s0[1] = 1, 2   # n in v0 and vr
        fr[3], sr[3] = 2, 2   # vr's n (label 3 of tNSns) from 2
        f1[1], s1[1] = 3, 1   # N in v1 and vr
        fr[1], sr[1] = 0, 1
    elif case == "xbox":
        f0[3] = f1[3] = 1
        s0[3] = s1[3] = 2
    elif case == "twrap":
        f0[0] = f1[0] = fr[0] = 3
        s0[0] = s1[0] = sr[0] = 2
    elif case == "all_t_in_r":
        f0[0] = f1[0] = 1
        s0[0] = s1[0] = sr[0] = 2
        fr[0] = 2
    ref = vr.copy()
    oracle_contraction(1.5 - 0.5j, "tnsxyzc", f0, s0, d0, False, v0, "tNSxyzc", f1, s1, d1, True,
                       v1, 0.5, "tNSns", fr, sr, dr, ref)
    out = _gpu_contraction(gpu, 1.5 - 0.5j, "tnsxyzc", f0, s0, d0, False, v0, "tNSxyzc", f1, s1,
                           d1, True, v1, 0.5, "tNSns", fr, sr, dr, vr.copy())
    assert rel_err(out, ref) < 1e-10
    untouched = np.ones(dr, bool)
    idx = [np.arange(f, f + s) % d for f, s, d in zip(fr, sr, dr)]
    untouched[np.ix_(*idx)] = False
    assert np.array_equal(out.reshape(dr)[untouched], vr.reshape(dr)[untouched])


@pytest.mark.parametrize("dtype,tol", [(np.complex128, 1e-10), (np.complex64, 2e-5)])
def test_split_groups_in_place(gpu, dtype, tol):
    """Label groups that are two runs of memory are contracted in place (no operand reorder):
    the chain's y^dagger y over x, y, z and color (K = XYZ + C, M = S + n, N = s + N in
    pXYZTSCn / pXYZTsCN) and the row-major lattice form tsxyzcn x tSxyzcN -> tNSns."""
    import torch
    import superbblas_amd as sb
    L, Lt, nc = 3, 4, 5
    dx = [1, L, L, L, Lt, 4, 3, nc]
    y = random_valued(_vol(dx), dtype, 41)
    dr = [Lt, 4, nc, 4, nc]
    ref = np.zeros(_vol(dr), dtype)
    z8, z5 = [0] * 8, [0] * 5
    oracle_contraction(1.0, "pXYZTSCn", z8, dx, dx, True, y, "pXYZTsCN", z8, dx, dx, False, y, 0.0,
                       "TSnsN", z5, dr, dr, ref)
    ty = torch.from_numpy(y).to(gpu)
    tr = torch.zeros(_vol(dr), dtype=ty.dtype, device=gpu)
    sb.timings_enable(True)
    sb.timings_reset()
    sb.contraction(1.0, _single(dx), z8, dx, dx, "pXYZTSCn", True, [ty], _single(dx), z8, dx, dx,
                   "pXYZTsCN", False, [ty], 0.0, _single(dr), z5, dr, dr, "TSnsN", [tr])
    torch.cuda.synchronize()
    copies = sb.timings_get("copy")[1]
    sb.timings_enable(False)
    assert copies == 0, "operands were reordered"
    assert rel_err(tr.cpu().numpy(), ref) < tol
    # row-major lattice contraction (dist.cpp:393-415)
    d0, d1, dr2 = _lattice(4, 3, "tsxyzcn", "tSxyzcN")
    v0 = random_valued(_vol(d0), dtype, 42)
    v1 = random_valued(_vol(d1), dtype, 43)
    ref2 = np.zeros(_vol(dr2), dtype)
    z7 = [0] * 7
    oracle_contraction(1.0, "tsxyzcn", z7, d0, d0, False, v0, "tSxyzcN", z7, d1, d1, False, v1,
                       0.0, "tNSns", z5, dr2, dr2, ref2)
    sb.timings_enable(True)
    sb.timings_reset()
    out = _gpu_contraction(gpu, 1.0, "tsxyzcn", z7, d0, d0, False, v0, "tSxyzcN", z7, d1, d1,
                           False, v1, 0.0, "tNSns", z5, dr2, dr2, np.zeros(_vol(dr2), dtype))
    copies = sb.timings_get("copy")[1]
    sb.timings_enable(False)
    assert copies == 0, "operands were reordered"
    assert rel_err(out, ref2) < tol
