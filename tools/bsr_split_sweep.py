#!/usr/bin/env python3
"""Sweep of the split-row 3x3 BSR kernel (bsr_ell9_split_kernel; config 3, 16^4, complex<double>,
x and y row major; not part of the product) against the row-chunk kernel: rhs columns per thread
(bsr.split_cw), nonzero blocks per thread (bsr.split_jb) and workgroup size (bsr.split_nt).
Every case is checked against the row-chunk kernel's output (relative max error) and timed with
the library's HIP-event timers.  One JSON line per case."""
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import superbblas_amd as sb  # noqa: E402


def lattice_op(sb, dev, L):
    V = L ** 4
    sites = np.array(np.unravel_index(np.arange(V), (L, L, L, L))).T
    jj = np.zeros((V, 9, 6), np.int32)
    jj[:, 0, :4] = sites
    k = 1
    for d in range(4):
        for s in (-1, 1):
            c = sites.copy()
            c[:, d] = (c[:, d] + s) % L
            jj[:, k, :4] = c
            k += 1
    dim = [L, L, L, L, 1, 3]
    full = [([0] * 6, dim)]
    vals = torch.randn(V * 81, dtype=torch.complex128, device=dev)
    return sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                         [torch.full((V,), 9, dtype=torch.int32, device=dev)],
                         [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])


def main():
    dev = torch.device("cuda:0")
    L = int(os.environ.get("L", "16"))
    V = L ** 4
    op = lattice_op(sb, dev, L)
    sb.tune_set("bsr.tile", 0)
    cws = [int(v) for v in os.environ.get("CW", "1,2,4").split(",")]
    jbs = [int(v) for v in os.environ.get("JB", "1,3,9").split(",")]
    nts = [int(v) for v in os.environ.get("NT", "256,512").split(",")]
    ilvs = [int(v) for v in os.environ.get("ILV", "1").split(",")]

    for ncols in [int(c) for c in os.environ.get("NCOLS", "4,8,12,16,24,32,64").split(",")]:
        dimx = [1, L, L, L, L, 1, 3, ncols]
        x = torch.randn(V * 3 * ncols, dtype=torch.complex128, device=dev)
        y = torch.empty_like(x)
        px = [([0] * 8, dimx)]

        def run():
            sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx, [x],
                          0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])

        def timed():
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
            return ms / calls / 1e3

        by = 16.0 * (81 * V + 2 * 3 * V * ncols) + 4.0 * (9 * V + V + 1)
        sb.tune_set("bsr.split_max_cols", 0)
        t = timed()
        ref = y.clone()
        print(json.dumps({"n": ncols, "kernel": "chunked", "kernel_us": round(t * 1e6, 2),
                          "frac_hbm": round(by / t / 8e12, 4)}), flush=True)
        for ilv in [int(v) for v in os.environ.get("ELL9_ILV", "").split(",") if v]:
            sb.tune_set("bsr.ell9_ilv", ilv)
            y.zero_()
            t = timed()
            err = float((y - ref).abs().max() / ref.abs().max())
            print(json.dumps({"n": ncols, "kernel": "chunked", "ilv": ilv,
                              "kernel_us": round(t * 1e6, 2), "frac_hbm": round(by / t / 8e12, 4),
                              "rel_err_vs_chunked": err}), flush=True)
        sb.tune_set("bsr.ell9_ilv", 2)
        sb.tune_set("bsr.split_max_cols", 1 << 20)
        for cw, jb, nt, ilv in itertools.product(cws, jbs, nts, ilvs):
            sb.tune_set("bsr.split_cw", cw)
            sb.tune_set("bsr.split_jb", jb)
            sb.tune_set("bsr.split_nt", nt)
            sb.tune_set("bsr.split_ilv", ilv)
            y.zero_()
            t = timed()
            err = float((y - ref).abs().max() / ref.abs().max())
            print(json.dumps({"n": ncols, "kernel": "split", "cw": cw, "jb": jb, "nt": nt,
                              "ilv": ilv,
                              "kernel_us": round(t * 1e6, 2), "frac_hbm": round(by / t / 8e12, 4),
                              "rel_err_vs_chunked": err}), flush=True)
        for k in ("bsr.split_cw", "bsr.split_jb", "bsr.split_nt"):
            sb.tune_set(k, 0)
        sb.tune_set("bsr.split_ilv", 2)
        sb.tune_set("bsr.split_max_cols", 32)
        del x, y, ref
    op.destroy()


if __name__ == "__main__":
    main()
