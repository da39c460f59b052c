"""The split-row 9-point 3x3 BSR kernel (kernels_bsr.hip bsr_ell9_split_kernel: one thread per
(block row, group of JB nonzero blocks, rhs lane), partial products summed through LDS in block
order; complex<double>, row-major x, the library's choice from 4 to 32 rhs columns) against the
oracle's builtin BSR loop (bsr.h:535-650): every (columns per thread, blocks per thread) form,
column counts that are not multiples of the lanes, lattices whose block-row count is not a
multiple of the workgroup's rows, the XCD part interleave, alpha / beta, column-major y, blocks
with column -1 (the split core / halo operator, tests/bsr.cpp:402-545) and a random pattern.
Integer-valued operators must match exactly; random ones within the rounding of a 27-term sum."""
import numpy as np
import pytest

from _common import T_CDOUBLE, oracle_bsr, rel_err
from _common import stencil_jj

pytestmark = pytest.mark.gpu


def run_split(gpu, dims, ncols, cw, jb, ilv=2, alpha=1.0, beta=0.0, y_layout="row", kind="stencil",
              cut=None, integer=False, seed=0, expect=2):
    import torch
    import superbblas_amd as sb
    rng = np.random.default_rng(seed)

    def vals_of(n):
        if integer:
            return (rng.integers(-4, 5, n) + 1j * rng.integers(-4, 5, n)).astype(np.complex128)
        return (rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)).astype(np.complex128)

    vol = int(np.prod(dims))
    jj = stencil_jj(dims, kind, rng, cut)
    ii = np.full(vol, 9, np.int32)
    vals = vals_of(vol * 81)
    dim = list(dims) + [1, 3]
    x = vals_of(vol * 3 * ncols)
    y0 = vals_of(vol * 3 * ncols)
    row = y_layout == "row"
    yref = y0 * beta if beta != 0 else np.zeros(vol * 3 * ncols, np.complex128)
    oracle_bsr(T_CDOUBLE, dim, 0, vol, 3, 3, ii, jj.reshape(-1), vals, False, x, ncols, True, yref,
               ncols if row else vol * 3, row, ncols, alpha, add=beta != 0)
    full = [([0] * 6, dim)]
    op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                       [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj.reshape(-1)).to(gpu)],
                       [torch.from_numpy(vals).to(gpu)])
    dimx = [1] + list(dims) + [1, 3, ncols]
    if row:
        oy, dimy = "pxyztscn", dimx
    else:
        oy, dimy = "pnxyztsc", [1, ncols] + list(dims) + [1, 3]
    keys = {"bsr.split_max_cols": 1 << 20, "bsr.row_max_cols": 0, "bsr.split_cw": cw,
            "bsr.split_jb": jb, "bsr.split_ilv": ilv}
    old = {k: sb.tune_get(k) for k in keys}
    try:
        for k, v in keys.items():
            sb.tune_set(k, v)
        ty = (torch.from_numpy(y0.copy()).to(gpu) if beta != 0
              else torch.zeros(vol * 3 * ncols, dtype=torch.complex128, device=gpu))
        sb.bsr_krylov(alpha, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTSCn", [0] * 8, dimx,
                      dimx, [torch.from_numpy(x).to(gpu)], beta, [([0] * 8, dimy)], oy, [0] * 8,
                      dimy, dimy, "p", [ty])
        torch.cuda.synchronize()
        used = sb.tune_get("bsr.last_kernel")
    finally:
        for k, v in old.items():
            sb.tune_set(k, v)
        op.destroy()
    assert used == expect, "kernel form %d ran, not %d" % (used, expect)
    err = rel_err(ty.cpu().numpy(), yref)
    if integer:
        assert err == 0.0
    else:
        assert err < 1e-13


@pytest.mark.parametrize("ncols", [4, 5, 12, 13, 24, 31])
@pytest.mark.parametrize("cw,jb", [(1, 3), (1, 9), (2, 3), (2, 9)])
def test_split_forms(gpu, ncols, cw, jb):
    # more than 256 threads per row: the launcher declines and the row-chunk kernel runs
    tpr = 9 // jb * -(-ncols // cw)
    run_split(gpu, (4, 4, 4, 4), ncols, cw, jb, integer=True, expect=2 if tpr <= 256 else 3)


@pytest.mark.parametrize("dims", [(3, 5, 4, 6), (2, 2, 2, 2), (5, 3, 7, 2)])
@pytest.mark.parametrize("ilv", [1, 2, 3])
def test_split_ragged_interleave(gpu, dims, ilv):
    """block-row counts that leave a partial last workgroup and XCD ranges of uneven length"""
    run_split(gpu, dims, 12, 2, 3, ilv=ilv)


@pytest.mark.parametrize("alpha,beta", [(0.5 - 2j, 0.0), (1.0, 1.0), (-1.5 + 0.5j, 2.0 - 1j)])
@pytest.mark.parametrize("y_layout", ["row", "col"])
@pytest.mark.parametrize("jb", [3, 9])
def test_split_alpha_beta_layout(gpu, alpha, beta, y_layout, jb):
    run_split(gpu, (4, 4, 4, 4), 12, 2, jb, alpha=alpha, beta=beta, y_layout=y_layout)


@pytest.mark.parametrize("ncols", [8, 24])
def test_split_cut_and_random(gpu, ncols):
    """column -1 blocks (the interior operator of the core / halo pair) and 9 random columns"""
    run_split(gpu, (4, 4, 4, 4), ncols, 2, 3, cut=4)
    run_split(gpu, (4, 4, 4, 4), ncols, 2, 3, kind="random", seed=5)


def test_split_default_choice(gpu):
    """the library picks the split kernel from 4 to 32 rhs columns (row-major x, complex<double>)"""
    import superbblas_amd as sb
    assert sb.tune_get("bsr.split_max_cols") == 32
    run_split(gpu, (4, 4, 4, 8), 12, 0, 0)
