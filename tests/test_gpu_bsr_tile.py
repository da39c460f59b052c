"""The lattice-tiled 9-point 3x3 BSR kernel (kernels_bsr.hip bsr_tile_kernel, plan: bsr.cpp
build_tile_plan; an opt-in, sbx_tune_set("bsr.tile", 1) before create_bsr) against the oracle's builtin BSR loop (bsr.h:535-650) and against the chunked
ELL kernels (sbx_tune_set("bsr.tile", 0): the row-chunk kernel and, up to 3 columns, the
one-thread-per-block kernel), on random-valued operators: lattices whose extents are
not multiples of the tile, every element type, 1..80 rhs columns (the tiled shapes and the
fallbacks around them; the tests lift the library's 8..16 column range), alpha / beta, column-major y, blocks with column -1 (the split core /
halo operator of tests/bsr.cpp:402-545) and a random (non-lattice) pattern whose rows exceed the
direct-entry budget.  The tiled kernel sums a row's direct (halo) blocks first, so the
tolerance is the rounding of a 27-term sum, not bit equality."""
import numpy as np
import pytest

from _common import T_CDOUBLE, T_CFLOAT, T_DOUBLE, T_FLOAT, oracle_bsr, rel_err

pytestmark = pytest.mark.gpu

TYPES = {"cdouble": (np.complex128, T_CDOUBLE, 1e-13), "cfloat": (np.complex64, T_CFLOAT, 2e-6),
         "double": (np.float64, T_DOUBLE, 1e-13), "float": (np.float32, T_FLOAT, 2e-6)}


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


def run_case(gpu, dims, ncols, tname, kind="stencil", alpha=1.0, beta=0.0, y_layout="row",
             cut=None, seed=0):
    import torch
    import superbblas_amd as sb
    dt, t, tol = TYPES[tname]
    rng = np.random.default_rng(seed)
    cplx = np.dtype(dt).kind == "c"

    def rand(n):
        r = rng.uniform(-1, 1, n)
        return (r + 1j * rng.uniform(-1, 1, n) if cplx else r).astype(dt)

    vol = int(np.prod(dims))
    jj = stencil_jj(dims, kind, rng, cut)
    ii = np.full(vol, 9, np.int32)
    vals = rand(vol * 81)
    dim = list(dims) + [1, 3]
    x = rand(vol * 3 * ncols)
    y0 = rand(vol * 3 * ncols)
    row = y_layout == "row"
    yref = y0.copy() if beta != 0 else np.zeros(vol * 3 * ncols, dt)
    if beta != 0:
        yref *= beta
    oracle_bsr(t, dim, 0, vol, 3, 3, ii, jj.reshape(-1), vals, False, x, ncols, True, yref,
               ncols if row else vol * 3, row, ncols, alpha, add=beta != 0)
    full = [([0] * 6, dim)]
    tt = {np.complex128: torch.complex128, np.complex64: torch.complex64,
          np.float64: torch.float64, np.float32: torch.float32}[dt]
    sb.tune_set("bsr.tile", 1)  # the plan is built by create_bsr while the tiled kernel is on
    op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                       [torch.from_numpy(ii).to(gpu)], [torch.from_numpy(jj.reshape(-1)).to(gpu)],
                       [torch.from_numpy(vals).to(gpu)])
    dimx = [1] + list(dims) + [1, 3, ncols]
    if row:
        oy, dimy = "pxyztscn", dimx
    else:
        oy, dimy = "pnxyztsc", [1, ncols] + list(dims) + [1, 3]
    outs = []
    sb.tune_set("bsr.tile_min_cols", 1)
    sb.tune_set("bsr.tile_max_cols", 1 << 20)
    try:
        for tile in (1, 0):
            sb.tune_set("bsr.tile", tile)
            ty = torch.from_numpy(y0.copy()).to(gpu) if beta != 0 else torch.zeros(
                vol * 3 * ncols, dtype=tt, device=gpu)
            sb.bsr_krylov(alpha, op, "xyztsc", "XYZTSC", [([0] * 8, dimx)], "pXYZTSCn", [0] * 8,
                          dimx, dimx, [torch.from_numpy(x).to(gpu)], beta, [([0] * 8, dimy)], oy,
                          [0] * 8, dimy, dimy, "p", [ty])
            torch.cuda.synchronize()
            outs.append(ty.cpu().numpy())
    finally:
        sb.tune_set("bsr.tile", 0)
        sb.tune_set("bsr.tile_min_cols", 8)
        sb.tune_set("bsr.tile_max_cols", 16)
        op.destroy()
    assert rel_err(outs[0], yref) < tol
    assert rel_err(outs[1], yref) < tol


@pytest.mark.parametrize("ncols", [1, 4, 12, 24, 48, 64, 80])
@pytest.mark.parametrize("tname", ["cdouble", "cfloat", "double", "float"])
def test_tile_lattice(gpu, ncols, tname):
    run_case(gpu, (4, 4, 4, 8), ncols, tname)


@pytest.mark.parametrize("dims", [(3, 5, 4, 6), (2, 2, 2, 2), (1, 4, 1, 8), (5, 3, 7, 2)])
@pytest.mark.parametrize("ncols", [4, 12, 33])
def test_tile_ragged_lattice(gpu, dims, ncols):
    """extents that are not multiples of the tile (partial tiles), size-1 and size-2 dims"""
    run_case(gpu, dims, ncols, "cdouble")


@pytest.mark.parametrize("alpha,beta", [(0.5 - 2j, 0.0), (1.0, 1.0), (-1.5 + 0.5j, 2.0 - 1j)])
@pytest.mark.parametrize("y_layout", ["row", "col"])
def test_tile_alpha_beta_layout(gpu, alpha, beta, y_layout):
    run_case(gpu, (4, 4, 4, 4), 12, "cdouble", alpha=alpha, beta=beta, y_layout=y_layout)


@pytest.mark.parametrize("ncols", [12, 64])
def test_tile_cut_columns(gpu, ncols):
    """the interior operator of the split core / halo pair: blocks crossing x = 0 or x = 3 read
    nothing (column -1)"""
    run_case(gpu, (4, 4, 4, 4), ncols, "cdouble", cut=4)


@pytest.mark.parametrize("ncols", [4, 12, 64])
def test_tile_random_pattern(gpu, ncols):
    """9 random columns per row: most are direct, rows past the direct budget stage the rest"""
    run_case(gpu, (4, 4, 4, 4), ncols, "cdouble", kind="random", seed=3)
