#!/usr/bin/env python3
"""BSR microbenchmark (not part of the product): config 3 (16^4 periodic 9-point stencil,
complex<double>) with 3x3 (spin 1 x color 3) and 12x12 (spin 4 x color 3) blocks, n rhs,
x pXYZTSCn (row major) -> y pxyztscn; kernel time from the library's HIP-event timers."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def run(L, spin, color, ncols, dev, reps=20):
    b = spin * color
    dim = [L, L, L, L, spin, color]
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
    ii = np.full(V, 9, np.int32)
    vals = torch.randn(V * 9 * b * b, dtype=torch.complex128, device=dev)
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, spin, color]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, False, [torch.from_numpy(ii).to(dev)],
                       [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])
    dimx = [1, L, L, L, L, spin, color, ncols]
    x = torch.randn(V * b * ncols, dtype=torch.complex128, device=dev)
    y = torch.empty_like(x)
    px = [([0] * 8, dimx)]

    def f():
        sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx, [x], 0.0,
                      px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])
    f()
    torch.cuda.synchronize()
    sb.timings_enable(True)
    sb.timings_reset()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    ms, calls = sb.timings_get("bsr")
    sb.timings_enable(False)
    op.destroy()
    t = ms / calls / 1e3
    by = 16.0 * (9 * b * b * V + 2 * b * V * ncols) + 4.0 * (9 * V + V + 1)
    return {"blocks": "%dx%d" % (b, b), "n": ncols, "us": round(t * 1e6, 1),
            "GBps": round(by / t / 1e9, 1), "GFLOPs": round(8.0 * 9 * b * b * V * ncols / t / 1e9, 1)}


def main():
    dev = torch.device("cuda:0")
    for spin in (1, 4):
        for n in (1, 12, 64):
            print(json.dumps(run(16, spin, 3, n, dev)))


if __name__ == "__main__":
    main()
