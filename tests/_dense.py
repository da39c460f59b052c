"""Layout helpers for the dense batched solvers (dense.h): the reference's working orders
(prepare_for_cholesky, dense.h:507-560; trsm/gesm 760-770) as numpy transposes, and the golden
inputs of oracle/ref_golden.cpp dense_cases.  Test infrastructure only."""
import numpy as np

from _golden import gen


def _labels(o, orows, ocols):
    ot = [c for c in o if c not in orows and c not in ocols]
    return ot


def to_matrices(v, o, dim, orows, ocols):
    """Tensor (labels o, SlowToFast) -> (nbatch, n, n) with [b, r, c], r / c the row / column
    indices in orows / ocols label order (last label fastest)."""
    ot = _labels(o, orows, ocols)
    order = ot + list(orows) + list(ocols)
    perm = [o.index(c) for c in order]
    a = v.reshape(dim).transpose(perm)
    n = int(np.prod([dim[o.index(c)] for c in orows]))
    return a.reshape(-1, n, n)


def from_matrices(m, o, dim, orows, ocols):
    ot = _labels(o, orows, ocols)
    order = ot + list(orows) + list(ocols)
    perm = [o.index(c) for c in order]
    shp = [dim[i] for i in perm]
    return m.reshape(shp).transpose(np.argsort(perm)).ravel()


def to_panel(v, o, dim, first, second):
    """Tensor -> (nbatch, A, B) with the labels `first` then `second` (batch labels: the rest,
    in o order)."""
    ot = [c for c in o if c not in first and c not in second]
    order = ot + list(first) + list(second)
    perm = [o.index(c) for c in order]
    a = v.reshape(dim).transpose(perm)
    na = int(np.prod([dim[o.index(c)] for c in first]))
    nb = int(np.prod([dim[o.index(c)] for c in second]))
    return a.reshape(-1, na, nb)


def from_panel(m, o, dim, first, second):
    ot = [c for c in o if c not in first and c not in second]
    order = ot + list(first) + list(second)
    perm = [o.index(c) for c in order]
    shp = [dim[i] for i in perm]
    return m.reshape(shp).transpose(np.argsort(perm)).ravel()


def dense_input(kind, nt, n, dtype, seed=3):
    """oracle/ref_golden.cpp dense_input: (nt, n, n) with [t, r, c]."""
    b = gen("int", nt * n * n, seed, dtype).reshape(nt, n, n)
    if kind == "hpd":
        a = np.einsum("tqr,tqc->trc", b.conj(), b) + n * np.eye(n)
    elif kind == "tri":
        a = np.full((nt, n, n), 99, dtype)
        iu = np.triu_indices(n, 1)
        a[:, iu[0], iu[1]] = b[:, iu[0], iu[1]]
        d = np.arange(n)
        a[:, d, d] = n + 3 + np.abs(b[:, d, d])
    else:
        a = b + 4 * n * np.eye(n)
    return a.astype(dtype)
