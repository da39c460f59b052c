#!/usr/bin/env python3
"""Gather-locality probe of the 9-point 3x3 BSR kernel (config 3 shape, 16^4, complex<double>;
not part of the product).  The operator keeps 9 blocks per row and the same value stream; only
the block columns change:
  stencil  -- the lattice 9-point stencil (the bench operator);
  self9    -- all 9 blocks read the row's own site (x gathers hit L1: the gather instruction
              count and latency without the L2/MALL traffic);
  tline    -- the site and t+-1..t+-4 (neighbours within 4 rows: L1/L2 hits);
  random   -- 9 random sites (no locality at all).
Prints one JSON line per (stencil, n) with the kernel time."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import superbblas_amd as sb  # noqa: E402


def columns(kind, L):
    V = L ** 4
    sites = np.array(np.unravel_index(np.arange(V), (L, L, L, L))).T
    jj = np.zeros((V, 9, 6), np.int32)
    if kind == "stencil":
        jj[:, 0, :4] = sites
        k = 1
        for d in range(4):
            for s in (-1, 1):
                c = sites.copy()
                c[:, d] = (c[:, d] + s) % L
                jj[:, k, :4] = c
                k += 1
    elif kind == "self9":
        jj[:, :, :4] = sites[:, None, :]
    elif kind == "tline":
        for k, s in enumerate((0, -1, 1, -2, 2, -3, 3, -4, 4)):
            c = sites.copy()
            c[:, 3] = (c[:, 3] + s) % L
            jj[:, k, :4] = c
    else:
        rng = np.random.default_rng(5)
        r = rng.integers(0, V, (V, 9))
        jj[:, :, :4] = sites[r]
    return jj


def main():
    dev = torch.device("cuda:0")
    if os.environ.get("ELL9"):
        sb.tune_set("bsr.ell9", int(os.environ["ELL9"]))
    if os.environ.get("TILE"):
        sb.tune_set("bsr.tile", int(os.environ["TILE"]))
    if os.environ.get("ROWMAX"):
        sb.tune_set("bsr.row_max_cols", int(os.environ["ROWMAX"]))
    if os.environ.get("ROWDMA"):
        sb.tune_set("bsr.row_dma", int(os.environ["ROWDMA"]))
    if os.environ.get("SLAB"):
        sb.tune_set("bsr.tile_slab", int(os.environ["SLAB"]))
    if os.environ.get("TROWS"):
        sb.tune_set("bsr.tile_rows", int(os.environ["TROWS"]))
    if os.environ.get("TILE_MIN"):
        sb.tune_set("bsr.tile_min_cols", int(os.environ["TILE_MIN"]))
        sb.tune_set("bsr.tile_max_cols", 1 << 20)
    L = 16
    V = L ** 4
    for kind in sys.argv[1:] or ("stencil", "self9", "tline", "random"):
        jj = columns(kind, L)
        dim = [L, L, L, L, 1, 3]
        full = [([0] * 6, dim)]
        vals = torch.randn(V * 81, dtype=torch.complex128, device=dev)
        op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                           [torch.full((V,), 9, dtype=torch.int32, device=dev)],
                           [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])
        for ncols in [int(c) for c in os.environ.get("NCOLS", "1,4,12,24,64").split(",")]:
            dimx = [1, L, L, L, L, 1, 3, ncols]
            x = torch.randn(V * 3 * ncols, dtype=torch.complex128, device=dev)
            y = torch.empty_like(x)
            px = [([0] * 8, dimx)]

            def run():
                sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx,
                              [x], 0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])
            run()
            torch.cuda.synchronize()
            sb.timings_enable(True)
            sb.timings_filter("bsr")
            sb.timings_reset()
            for _ in range(10):
                run()
            torch.cuda.synchronize()
            ms, calls = sb.timings_get("bsr")
            sb.timings_enable(False)
            sb.timings_filter(None)
            t = ms / calls / 1e3
            by = 16.0 * (81 * V + 2 * 3 * V * ncols) + 4.0 * (9 * V + V + 1)
            print(json.dumps({"stencil": kind, "tile": os.environ.get("TILE", "default"),
                              "slab": os.environ.get("SLAB", "default"),
                              "row_max": os.environ.get("ROWMAX", "default"),
                              "row_dma": os.environ.get("ROWDMA", "default"),
                              "rows": os.environ.get("TROWS", "16"),
                              "n": ncols, "kernel_us": round(t * 1e6, 2),
                              "frac_hbm": round(by / t / 8e12, 4)}), flush=True)
        op.destroy()


if __name__ == "__main__":
    main()
