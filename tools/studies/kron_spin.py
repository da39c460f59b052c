#!/usr/bin/env python3
"""Kronecker BSR (bench `kron_n12`: 16^4 sites, 3x3 color blocks x the Wilson 4x4 spin matrices,
complex<double>): the spin-first VALU kernel (bsr.kron_spin 1, bsr_kron_spin_kernel) with and
without the XCD row order (bsr.kron_order) against the MFMA kernels (bsr.kron_spin 0).
VARIANTS=spin:order,...; NCOLS=12,...; KINDS=stencil,self (tools/studies/bsr_bound.py's
column kinds: `self` points all nine neighbours at the row's own site, a traffic floor).
Variants interleaved over ROUNDS, warm; kernel time from the library's HIP-event timers;
the spin-first forms must agree bit for bit, and with the MFMA form to rounding.  Not part of
the product."""
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402
from bsr_bound import columns  # noqa: E402
from kron_bound import spin_matrices  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    L = int(os.environ.get("L", "16"))
    V = L ** 4
    kinds = os.environ.get("KINDS", "stencil").split(",")
    ncols_list = [int(v) for v in os.environ.get("NCOLS", "12").split(",")]
    variants = [tuple(int(x) for x in v.split(":"))
                for v in os.environ.get("VARIANTS", "2:1,2:0,1:1,0:1").split(",")]
    rounds = int(os.environ.get("ROUNDS", "3"))
    dims = [L, L, L, L]
    dim = dims + [4, 3]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 4, 1]
    ks = spin_matrices()
    g = torch.Generator(device=dev).manual_seed(7)
    for kind in kinds:
        jj, nnz = columns(kind, (L, L, L, L))
        kron = torch.from_numpy(ks[:nnz].reshape(-1)).to(dev)
        cvals = torch.randn(V * nnz * 9, dtype=torch.complex128, device=dev, generator=g)
        op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, False,
                                [torch.full((V,), nnz, dtype=torch.int32, device=dev)],
                                [torch.from_numpy(jj.reshape(-1)).to(dev)], [cvals], [kron])
        for n in ncols_list:
            dimx = [1] + dims + [3, n, 4]
            px = [([0] * 8, dimx)]
            x = torch.randn(V * 12 * n, dtype=torch.complex128, device=dev, generator=g)
            y = torch.empty_like(x)

            def f():
                sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTCnS", [0] * 8, dimx, dimx,
                              [x], 0.0, px, "pxyztcns", [0] * 8, dimx, dimx, "p", [y])
            times = {v: [] for v in variants}
            outs, forms = {}, {}
            for _ in range(rounds):
                for v in variants:
                    sb.tune_set("bsr.kron_spin", v[0])
                    sb.tune_set("bsr.kron_order", v[1])
                    for _ in range(10):
                        f()
                    torch.cuda.synchronize()
                    sb.timings_enable(True)
                    sb.timings_filter("bsr")
                    sb.timings_reset()
                    for _ in range(20):
                        f()
                    torch.cuda.synchronize()
                    ms, calls = sb.timings_get("bsr")
                    sb.timings_enable(False)
                    times[v].append(ms / calls / 1e3)
                    forms[v] = sb.tune_get("bsr.last_kernel")
                    outs[v] = y.clone()
            sb.tune_set("bsr.kron_spin", 0)
            sb.tune_set("bsr.kron_order", 1)
            algo = 16.0 * (81 * V + 2 * 12 * V * n) + 4.0 * 9 * V  # the stencil's
            base = outs[variants[0]]
            scale = float(base.abs().max())
            for v in variants:
                t = statistics.median(times[v])
                print(json.dumps({"kind": kind, "ncols": n, "spin_first": v[0], "xcd_order": v[1],
                                  "kernel": forms[v], "us": round(t * 1e6, 1),
                                  "us_min": round(min(times[v]) * 1e6, 1),
                                  "stencil_bytes_frac_hbm": round(algo / t / 8e12, 4),
                                  "maxdiff_vs_first": float((outs[v] - base).abs().max()) / scale}),
                      flush=True)
            del x, y
        op.destroy()
        del cvals


if __name__ == "__main__":
    main()
