#!/usr/bin/env python3
"""Bound model of the Kronecker BSR kernel (bench `kron_n12`: 16^4, 3x3 color blocks x 4x4 spin
matrices, complex<double>): the same kernel and launch on operators that differ only in where
the nine block columns of a row point (tools/studies/bsr_bound.py's kinds: stencil, local, self, one),
so the value, y and gather streams stay fixed while the x reuse distance changes.  XLS=3,2,1,0: the
bsr.kron_xlds settings to compare (x staged by LDS-DMA that many neighbours ahead, or per lane);
YL=1: y through the same ring (bsr.kron_ylds).  Not part of the
product."""
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402
from bsr_bound import columns  # noqa: E402


def spin_matrices():
    i_ = 1j
    g = [np.array([[0, 0, 0, i_], [0, 0, i_, 0], [0, -i_, 0, 0], [-i_, 0, 0, 0]]),
         np.array([[0, 0, 0, -1], [0, 0, 1, 0], [0, 1, 0, 0], [-1, 0, 0, 0]]),
         np.array([[0, 0, i_, 0], [0, 0, 0, -i_], [-i_, 0, 0, 0], [0, i_, 0, 0]]),
         np.array([[0, 0, 1, 0], [0, 0, 0, 1], [1, 0, 0, 0], [0, 1, 0, 0]])]
    ks = [np.eye(4)]
    for gm in g:
        ks += [np.eye(4) - gm, np.eye(4) + gm]
    return np.array(ks, np.complex128)


def main():
    dev = torch.device("cuda:0")
    L = int(os.environ.get("L", "16"))
    V = L ** 4
    kinds = os.environ.get("KINDS", "stencil,local,self,one").split(",")
    ncols_list = [int(v) for v in os.environ.get("NCOLS", "12").split(",")]
    xls = [int(v) for v in os.environ.get("XLS", str(sb.tune_get("bsr.kron_xlds"))).split(",")]
    sb.tune_set("bsr.kron_ylds", int(os.environ.get("YL", sb.tune_get("bsr.kron_ylds"))))
    dims = [L, L, L, L]
    dim = dims + [4, 3]
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 4, 1]
    ks = spin_matrices()
    for kind in kinds:
        jj, nnz = columns(kind, (L, L, L, L))
        kron = torch.from_numpy(ks[:nnz].reshape(-1)).to(dev)
        cvals = torch.randn(V * nnz * 9, dtype=torch.complex128, device=dev)
        op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, False,
                                [torch.full((V,), nnz, dtype=torch.int32, device=dev)],
                                [torch.from_numpy(jj.reshape(-1)).to(dev)], [cvals], [kron])
        for n, xl in [(n, xl) for n in ncols_list for xl in xls]:
            sb.tune_set("bsr.kron_xlds", xl)
            dimx = [1] + dims + [3, n, 4]
            px = [([0] * 8, dimx)]
            x = torch.randn(V * 12 * n, dtype=torch.complex128, device=dev)
            y = torch.empty_like(x)

            def f():
                sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTCnS", [0] * 8, dimx, dimx,
                              [x], 0.0, px, "pxyztcns", [0] * 8, dimx, dimx, "p", [y])
            for _ in range(30):
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
            algo = 16.0 * (81 * V + 2 * 12 * V * n) + 4.0 * 9 * V  # the stencil's
            floor = 16.0 * (nnz * 9 * V + 2 * 12 * V * n) + 4.0 * nnz * V
            print(json.dumps({"kind": kind, "ncols": n, "xlds": xl, "us": round(t * 1e6, 1),
                              "kernel": sb.tune_get("bsr.last_kernel"),
                              "stencil_bytes_frac_hbm": round(algo / t / 8e12, 4),
                              "min_bytes_MB": round(floor / 1e6, 1),
                              "min_bytes_TBps": round(floor / t / 1e12, 2)}), flush=True)
            del x, y
        op.destroy()
        del cvals
    sb.tune_set("bsr.kron_xlds", xls[0])


if __name__ == "__main__":
    main()
