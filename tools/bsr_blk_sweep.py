#!/usr/bin/env python3
"""12x12 (spin x color) 9-point BSR: the block-staged MFMA kernel with register staging
(bsr.blk_dma 0) against LDS-DMA staging one or two blocks ahead (1 / 2); 16^4 complex<double>
and the chain's 16^3 x 64 complex<float> operator, n = 12, x / y row major.  Outputs must be
bit-identical (same products, same order).  The GPU is brought to clock first (0.5 s of the
kernel), then the modes are timed round-robin (ROUNDS passes; min and median), since the clocks
drift by ~10 % over the first seconds.  One JSON line per case (not part of the product)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import superbblas_amd as sb  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for dims, dt in (((16, 16, 16, 16), torch.complex128), ((16, 16, 16, 64), torch.complex64)):
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
        dim = list(dims) + [4, 3]
        full = [([0] * 6, dim)]
        vals = torch.randn(V * 9 * 144, dtype=dt, device=dev)
        if os.environ.get("VALS") == "int":  # small integers: fewer toggling mantissa bits
            vals = torch.randint(-2, 3, (V * 9 * 144,), device=dev).to(dt)
        op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 4, 3], [1, 1, 1, 1, 4, 3], False,
                           [torch.full((V,), 9, dtype=torch.int32, device=dev)],
                           [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])
        ncols = int(os.environ.get("NCOLS", "12"))
        dimx = [1] + list(dims) + [4, 3, ncols]
        x = torch.randn(V * 12 * ncols, dtype=dt, device=dev)
        if os.environ.get("VALS") == "int":
            x = torch.randint(-2, 3, (V * 12 * ncols,), device=dev).to(dt)
        y = torch.empty_like(x)
        px = [([0] * 8, dimx)]
        es = x.element_size()
        by = es * (9 * 144 * V + 2 * 12 * V * ncols) + 4.0 * (9 * V + V + 1)
        ref = None
        # mode 10 + d: blocks staged d ahead with packed slots (bsr.blk_pack 1); d: 1-KB-rounded
        modes = [int(m) for m in os.environ.get("MODES", "0,1,2,11").split(",")]

        def set_mode(mode):
            sb.tune_set("bsr.blk_dma", mode % 10)
            sb.tune_set("bsr.blk_pack", 2 if mode >= 10 else 0)

        def run():
            sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx, [x],
                          0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])
        # clocks up first (~0.5 s of the kernel), then the modes round-robin, min and median
        set_mode(modes[0])
        t0 = time.time()
        while time.time() - t0 < 0.5:
            run()
            torch.cuda.synchronize()
        times = {m: [] for m in modes}
        same = {}
        for _ in range(int(os.environ.get("ROUNDS", "4"))):
            for mode in modes:
                set_mode(mode)
                run()
                torch.cuda.synchronize()
                if ref is None:
                    ref = y.clone()
                same[mode] = bool(torch.equal(y, ref))
                sb.timings_enable(True)
                sb.timings_filter("bsr")
                sb.timings_reset()
                for _ in range(10):
                    run()
                torch.cuda.synchronize()
                ms, calls = sb.timings_get("bsr")
                sb.timings_enable(False)
                sb.timings_filter(None)
                times[mode].append(ms / calls / 1e3)
        for mode in modes:
            t = min(times[mode])
            print(json.dumps({"dims": dims, "dtype": str(dt).split(".")[-1], "n": ncols,
                              "blk_dma": mode, "kernel_us_min": round(t * 1e6, 1),
                              "kernel_us_median": round(float(np.median(times[mode])) * 1e6, 1),
                              "GBps": round(by / t / 1e9, 1), "frac_hbm": round(by / t / 8e12, 4),
                              "same_as_first": same[mode]}), flush=True)
        sb.tune_set("bsr.blk_dma", -1)
        sb.tune_set("bsr.blk_pack", 1)
        op.destroy()
        del x, y, vals, ref


if __name__ == "__main__":
    main()
