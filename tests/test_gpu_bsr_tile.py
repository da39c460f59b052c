"""The site-tile 9-point 3x3 BSR kernel (kernels_bsr.hip bsr_ell9_tile_kernel: the rows grouped
into 2x2x2x2 site tiles by the operator's schedule, bsr.cpp build_tile_schedule; a tile's distinct
x rows staged in LDS per slice of 8 rhs columns, its values once; complex<double>, row-major x and
y, opt-in through bsr.tile, from 33 rhs columns) against the oracle's builtin BSR loop (bsr.h:535-650):
column counts, lattices whose extents are odd or smaller than a tile (ragged tiles), alpha / beta,
blocks with column -1 (the core / halo split, tests/bsr.cpp:402-545), a random pattern (tiles with
many distinct columns), and the shapes it declines (column-major y, a column count that is not a
multiple of 8, the tune key off).  Integer-valued operators must match exactly; random ones
within the rounding of a 27-term sum."""
import numpy as np
import pytest

from _common import T_CDOUBLE, oracle_bsr, rel_err
from _common import stencil_jj

pytestmark = pytest.mark.gpu

TILE, ROWS = 4, 3  # bsr.last_kernel: site tiles, row chunks
# (bsr.tile form, bsr.last_kernel): 16-site tiles with slices of 8 columns, 8-site tiles with
# slices of 16 columns (round 6: no LDS bank conflicts whatever the slots)
FORMS = [(1, TILE), (2, 13)]
FORM_IDS = ["tile16x8", "tile8x16"]


def run_tile(gpu, dims, ncols, alpha=1.0, beta=0.0, y_layout="row", kind="stencil", cut=None,
             integer=False, seed=0, expect=TILE, tile=1):
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
    old = sb.tune_get("bsr.tile")
    try:
        sb.tune_set("bsr.tile", tile)
        ty = (torch.from_numpy(y0.copy()).to(gpu) if beta != 0
              else torch.zeros(vol * 3 * ncols, dtype=torch.complex128, device=gpu))
        sb.bsr_krylov(alpha, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTSCn", [0] * 8, dimx,
                      dimx, [torch.from_numpy(x).to(gpu)], beta, [([0] * 8, dimy)], oy, [0] * 8,
                      dimy, dimy, "p", [ty])
        torch.cuda.synchronize()
        used = sb.tune_get("bsr.last_kernel")
    finally:
        sb.tune_set("bsr.tile", old)
        op.destroy()
    assert expect is None or used == expect, "kernel form %d ran, not %d" % (used, expect)
    err = rel_err(ty.cpu().numpy(), yref)
    if integer:
        assert err == 0.0
    else:
        assert err < 1e-13


@pytest.mark.parametrize("form", FORMS, ids=FORM_IDS)
@pytest.mark.parametrize("ncols", [40, 64, 128])
def test_tile_columns(gpu, ncols, form):
    tile, kern = form
    ns = 8 if tile == 1 else 16
    run_tile(gpu, (4, 4, 4, 4), ncols, integer=True, tile=tile,
             expect=kern if ncols % ns == 0 else ROWS)


@pytest.mark.parametrize("dims", [(3, 5, 4, 6), (2, 2, 2, 2), (5, 3, 7, 2), (1, 1, 4, 9), (6, 6, 6, 6)])
@pytest.mark.parametrize("form", FORMS, ids=FORM_IDS)
def test_tile_ragged_lattices(gpu, dims, form):
    """extents that leave partial tiles, and lattices with fewer than four extended dims"""
    run_tile(gpu, dims, 64, tile=form[0], expect=form[1])


@pytest.mark.parametrize("alpha,beta", [(0.5 - 2j, 0.0), (1.0, 1.0), (-1.5 + 0.5j, 2.0 - 1j)])
@pytest.mark.parametrize("form", FORMS, ids=FORM_IDS)
def test_tile_alpha_beta(gpu, alpha, beta, form):
    run_tile(gpu, (4, 4, 4, 8), 48, alpha=alpha, beta=beta, tile=form[0], expect=form[1])


@pytest.mark.parametrize("form", FORMS, ids=FORM_IDS)
def test_tile_cut_and_random(gpu, form):
    """column -1 blocks (the interior operator of the core / halo pair) and 9 random columns"""
    run_tile(gpu, (4, 4, 4, 4), 64, cut=4, integer=True, tile=form[0], expect=form[1])
    run_tile(gpu, (4, 4, 4, 4), 64, kind="random", seed=5, expect=None, tile=form[0])


def test_tile_declined_shapes(gpu):
    """column-major y, a column count that is not a multiple of 8, the tune key off: the row-chunk
    kernel runs instead, with the same results"""
    run_tile(gpu, (4, 4, 4, 4), 64, y_layout="col", expect=ROWS)
    run_tile(gpu, (4, 4, 4, 4), 44, expect=ROWS)
    run_tile(gpu, (4, 4, 4, 4), 64, tile=0, expect=ROWS)
    run_tile(gpu, (4, 4, 4, 4), 40, tile=2, expect=ROWS)  # 16-column slices: 40 declined


def test_tile_default_choice(gpu):
    """opt-in (bsr.tile 1): by default the row-chunk kernel runs at 64 columns (the site tiles
    measured slower on the config-3 shape); with the key on they run from 33"""
    import superbblas_amd as sb
    assert sb.tune_get("bsr.tile") == 0 and sb.tune_get("bsr.tile_min_cols") == 33
    run_tile(gpu, (8, 8, 8, 8), 64, integer=True, tile=0, expect=ROWS)
    run_tile(gpu, (8, 8, 8, 8), 64, integer=True)
    run_tile(gpu, (8, 8, 8, 8), 64, integer=True, tile=2, expect=13)
