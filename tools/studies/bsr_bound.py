#!/usr/bin/env python3
"""Bound model of the 3x3-block 9-point BSR kernel (config 3, 16^4, complex<double>): the same
kernel and launch on operators that differ only in WHERE the nine block columns of a row point,
so the value stream, the y stream and the number of x-row gathers per row stay fixed while the x
reuse distance changes.  Not part of the product.

  stencil  the 9-point stencil (self, +-x, +-y, +-z, +-t; +-x is 4096 sites away)
  local    the same count of gathers, all nine within +-4 sites of the row (reuse distance
           ~ 4 rows: every repeat fetch is an L2 (mostly L1) hit -- the fabric/HBM floor of x)
  self     all nine columns the row's own site (one distinct x row per row)
  one      a single nonzero block per row (the own site; 1/9 of the values and gathers)

Printed per case and rhs count: kernel time (library timers, median of 3 rounds of 20
launches), the stencil's algorithmic bytes / time as a fraction of 8 TB/s, and the bytes the
case must move beyond L2 at the least (values + y + indices + x once).  DIMS=16,16,16,64: the lattice (default L^4, L=16).  VARIANTS / REGS / TILES: bsr.variant /
bsr.reg / bsr.tile values to compare.  BLK=12 / DT=cf: the
12x12-block (spin 4 x color 3) operator, complex<float>.  NTS=0,1,...: the bsr.nt settings to
compare (the value stream's non-temporal load policy, per kernel bit); PDS=1,2,3: the 12x12
kernel's block lookahead (bsr.blk_pd)."""
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def columns(kind, L):
    V = int(np.prod(L))
    sites = np.array(np.unravel_index(np.arange(V), tuple(L))).T
    if kind == "one":
        jj = np.zeros((V, 1, 6), np.int32)
        jj[:, 0, :4] = sites
        return jj, 1
    jj = np.zeros((V, 9, 6), np.int32)
    jj[:, 0, :4] = sites
    k = 1
    for d in range(4):
        for s in (-1, 1):
            c = sites.copy()
            if kind == "stencil":
                c[:, d] = (c[:, d] + s) % L[d]
            elif kind == "local":
                c[:, 3] = (c[:, 3] + s * (d + 1)) % L[3]  # t +- 1..4: rows +- 1..4
            jj[:, k, :4] = c
            k += 1
    return jj, 9


def main():
    dev = torch.device("cuda:0")
    L = [int(v) for v in os.environ.get("DIMS", ",".join([os.environ.get("L", "16")] * 4)).split(",")]
    V = int(np.prod(L))
    kinds = os.environ.get("KINDS", "stencil,local,self,one").split(",")
    ncols_list = [int(v) for v in os.environ.get("NCOLS", "12,64").split(",")]
    nts = [int(v) for v in os.environ.get("NTS", str(sb.tune_get("bsr.nt"))).split(",")]
    pds = [int(v) for v in os.environ.get("PDS", str(sb.tune_get("bsr.blk_pd"))).split(",")]
    variants = [int(v) for v in os.environ.get("VARIANTS", str(sb.tune_get("bsr.variant"))).split(",")]
    regs = [int(v) for v in os.environ.get("REGS", "-1").split(",")]
    # (VREGS / STREAMS: the round-6 bsr.vreg / bsr.stream experiments, removed again: commit ad3532b)
    tiles = [int(v) for v in os.environ.get("TILES", str(sb.tune_get("bsr.tile"))).split(",")]
    # BLK=12: spin 4 x color 3 blocks (config 3's secondary shape / the chain's operator);
    # DT=cf: complex<float>
    spin = 4 if os.environ.get("BLK", "3") == "12" else 1
    dt = torch.complex64 if os.environ.get("DT", "cd") == "cf" else torch.complex128
    es = 8 if dt == torch.complex64 else 16
    b = 3 * spin
    dim = L + [spin, 3]
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, spin, 3]
    for kind in kinds:
        jj, nnz = columns(kind, L)
        vals = torch.randn(V * nnz * b * b, dtype=dt, device=dev)
        op = sb.create_bsr(full, dim, full, dim, blk, blk, False,
                           [torch.full((V,), nnz, dtype=torch.int32, device=dev)],
                           [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])
        for n, nt, pd, var, reg, tile in [(n, nt, pd, var, reg, tile) for n in ncols_list for nt in nts
                                          for pd in pds for var in variants for reg in regs
                                          for tile in tiles]:
            sb.tune_set("bsr.tile", tile)
            sb.tune_set("bsr.variant", var)
            if reg >= 0:  # bsr.reg: the round-5 register-staged experiment (removed again)
                sb.tune_set("bsr.reg", reg)
            sb.tune_set("bsr.nt", nt)
            sb.tune_set("bsr.blk_pd", pd)
            dx = [1] + L + [spin, 3, n]
            px = [([0] * 8, dx)]
            x = torch.randn(V * b * n, dtype=dt, device=dev)
            y = torch.empty_like(x)

            def f():
                sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dx, dx, [x],
                              0.0, px, "pxyztscn", [0] * 8, dx, dx, "p", [y])
            for _ in range(30):  # warm clocks
                f()
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                sb.timings_enable(True)
                sb.timings_reset()
                for _ in range(20):
                    f()
                torch.cuda.synchronize()
                ms, calls = sb.timings_get("bsr")
                sb.timings_enable(False)
                ts.append(ms / calls / 1e3)
            t = statistics.median(ts)
            algo = es * (9 * b * b * V + 2 * b * V * n) + 4.0 * (9 * V + V + 1)  # the stencil's
            floor = es * (nnz * b * b * V + 2 * b * V * n) + 4.0 * (nnz * V + V + 1)
            print(json.dumps({"blk": b, "dtype": str(dt), "kind": kind, "ncols": n, "nt": nt, "blk_pd": pd, "variant": var, "reg": reg, "tile": tile,
                              "us": round(t * 1e6, 1),
                              "kernel": sb.tune_get("bsr.last_kernel"),
                              "stencil_bytes_frac_hbm": round(algo / t / 8e12, 4),
                              "min_bytes_MB": round(floor / 1e6, 1),
                              "min_bytes_TBps": round(floor / t / 1e12, 2)}), flush=True)
            del x, y
        op.destroy()
        del vals


if __name__ == "__main__":
    main()
