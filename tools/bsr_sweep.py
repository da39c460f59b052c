#!/usr/bin/env python3
"""Shape sweep of the 9-point 3x3 BSR kernel (config 3, 16^4, complex<double>; not part of the
product): sbx_tune_set("bsr.ell9", variant) x ("bsr.ell9_lds", bytes) at n = 1 / 12 / 64.
Every variant's output must equal the default kernel's bit for bit (same summation order).
Prints one JSON line per case with the kernel time (library HIP-event timers)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import superbblas_amd as sb  # noqa: E402

VARIANTS = {0: "nt256 pd1 g2", 1: "nt64 pd1 g2", 2: "nt128 pd1 g2", 3: "nt64 pd2 g2",
            4: "nt128 pd2 g2", 5: "nt64 pd1 g1", 6: "nt128 pd2 g1", 7: "nt256 pd2 g2",
            8: "nt256 pd1 g2 ntY", 9: "nt256 pd1 g2 ntV", 10: "nt256 pd1 g2 ntVY",
            11: "nt256 pd2 g2 ntY", 12: "nt256 pd2 g2 ntVY",
            13: "nt256 pd1 g2 sc", 14: "nt256 pd2 g2 sc", 15: "nt256 pd1 g4 sc",
            16: "nt256 pd1 g2 dma", 17: "nt256 pd2 g2 dma", 18: "nt256 pd1 g2 sc dma"}


def main():
    dev = torch.device("cuda:0")
    L = 16
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
    op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                       [torch.full((V,), 9, dtype=torch.int32, device=dev)],
                       [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])
    sb.tune_set("bsr.tile", 0)
    sb.tune_set("bsr.row_max_cols", 0)
    for ncols in [int(c) for c in os.environ.get("NCOLS", "1,12,64").split(",")]:
        dimx = [1, L, L, L, L, 1, 3, ncols]
        x = torch.randn(V * 3 * ncols, dtype=torch.complex128, device=dev)
        y = torch.empty_like(x)
        px = [([0] * 8, dimx)]

        def run():
            sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx, [x],
                          0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])
        ref = None
        by = 16.0 * (81 * V + 2 * 3 * V * ncols) + 4.0 * (9 * V + V + 1)
        vs = [int(v) for v in os.environ.get("VARIANTS", "").split(",") if v] or list(VARIANTS)
        ls = [int(v) for v in os.environ.get("LDS", "0,6144,12288,24576,49152").split(",")]
        for var, lds in [(v, l) for v in [0] + [v for v in vs if v != 0] for l in ls]:
            sb.tune_set("bsr.ell9", var)
            sb.tune_set("bsr.ell9_lds", lds)
            try:
                run()
                torch.cuda.synchronize()
            except Exception as e:  # a shape the variant cannot take
                print(json.dumps({"n": ncols, "variant": VARIANTS[var], "lds": lds,
                                  "error": str(e)[:100]}), flush=True)
                continue
            if ref is None:
                ref = y.clone()
            same = bool(torch.equal(y, ref))
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
            print(json.dumps({"n": ncols, "variant": VARIANTS[var], "lds": lds,
                              "kernel_us": round(t * 1e6, 2), "frac_hbm": round(by / t / 8e12, 4),
                              "same_as_default": same}), flush=True)
        sb.tune_set("bsr.ell9", 0)
        sb.tune_set("bsr.ell9_lds", 0)
    op.destroy()


if __name__ == "__main__":
    main()
