#!/usr/bin/env python3
"""12x12-block BSR kernel variants (not part of the product): config 3's secondary shape
(16^4, spin 4 x color 3, complex<double>, n = 12) and the chain's operator (16^3 x 64,
complex<float>, n = 12): the library's kernel (variant 0) against the round-1 kernel (variant 1,
sbx_tune_set("bsr.variant")); results checked equal."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def op_and_vectors(dims, spin, color, ncols, dtype, dev):
    b = spin * color
    V = int(np.prod(dims))
    sites = np.array(np.unravel_index(np.arange(V), dims)).T
    jj = np.zeros((V, 9, 6), np.int32)
    jj[:, 0, :4] = sites
    k = 1
    for d in range(4):
        for s in (-1, 1):
            c = sites.copy()
            c[:, d] = (c[:, d] + s) % dims[d]
            jj[:, k, :4] = c
            k += 1
    vals = torch.randn(V * 9 * b * b, dtype=dtype, device=dev)
    dim = list(dims) + [spin, color]
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, spin, color]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, False,
                       [torch.full((V,), 9, dtype=torch.int32, device=dev)],
                       [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])
    dimx = [1] + list(dims) + [spin, color, ncols]
    x = torch.randn(V * b * ncols, dtype=dtype, device=dev)
    y = torch.empty_like(x)
    return op, x, y, dimx, V, b


def main():
    dev = torch.device("cuda:0")
    for name, dims, dtype, spin, ncols in (
            ("16^4 cdouble 3x3 n=1", (16, 16, 16, 16), torch.complex128, 1, 1),
            ("16^4 cdouble 3x3 n=4", (16, 16, 16, 16), torch.complex128, 1, 4),
            ("16^4 cdouble 3x3", (16, 16, 16, 16), torch.complex128, 1, 12),
            ("16^4 cdouble 3x3 n=64", (16, 16, 16, 16), torch.complex128, 1, 64),
            ("16^4 cdouble", (16, 16, 16, 16), torch.complex128, 4, 12),
            ("16^3x64 cfloat", (16, 16, 16, 64), torch.complex64, 4, 12)):
        op, x, y, dimx, V, b = op_and_vectors(dims, spin, 3, ncols, dtype, dev)
        px = [([0] * 8, dimx)]
        es = 16 if dtype == torch.complex128 else 8

        def f():
            sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx, [x],
                          0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])
        ref = None
        for var in ((1, 0) if spin == 1 else (1, 2, 0)):
            sb.tune_set("bsr.variant", var)
            f()
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            err = float((y - ref).abs().max() / ref.abs().max())
            sb.timings_enable(True)
            sb.timings_reset()
            for _ in range(20):
                f()
            torch.cuda.synchronize()
            ms, calls = sb.timings_get("bsr")
            sb.timings_enable(False)
            t = ms / calls / 1e3
            by = es * (9 * b * b * V + 2 * b * V * ncols) + 4.0 * (9 * V + V + 1)
            print(json.dumps({"case": name, "variant": var, "us": round(t * 1e6, 1),
                              "GBps": round(by / t / 1e9, 1), "rel_err_vs_v0": err}), flush=True)
        sb.tune_set("bsr.variant", 0)
        op.destroy()


if __name__ == "__main__":
    main()
