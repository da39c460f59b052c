#!/usr/bin/env python3
"""Config-2 GEMM (16^4, n = 64, complex<double>): who issues the slab DMA (not part of the product;
sbx_tune_set("gemm.loaders" / "gemm.dma_spread")).  Every wave its share (0), or only waves 0..LW-1
(LW = 4 / 8 / 16) spreading it over SP k-steps.  Variants interleaved over several rounds, warm;
GEMM kernel time from the library's HIP-event timers; results must be bit-identical."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402

VARIANTS = [tuple(int(x) for x in v.split(":")) for v in
            os.environ.get("VARIANTS", "0:1,4:1,4:4,8:1,8:4,16:4").split(",")]  # loaders:spread[:nt]


def main():
    dev = torch.device("cuda:0")
    L, n = 16, 64
    d0 = [L, n, 4, L, L, L, 3]
    dr = [L, n, 4, n, 4]
    vol0 = 1
    for x in d0:
        vol0 *= x
    g = torch.Generator(device=dev).manual_seed(5)
    v0 = torch.randn(vol0, dtype=torch.complex128, device=dev, generator=g)
    v1 = torch.randn(vol0, dtype=torch.complex128, device=dev, generator=g)
    vr = torch.zeros(L * n * 4 * n * 4, dtype=torch.complex128, device=dev)
    z7, z5 = [0] * 7, [0] * 5
    flops = 8.0 * L * (L ** 3 * 3) * (n * 4) ** 2

    def step():
        sb.contraction(1.0, [(z7, d0)], z7, d0, d0, "tnsxyzc", False, [v0], [(z7, d0)], z7, d0,
                       d0, "tNSxyzc", False, [v1], 0.0, [(z5, dr)], z5, dr, dr, "tNSns", [vr])

    ref = None
    times = {v: [] for v in VARIANTS}
    for _ in range(30):  # clocks up
        step()
    torch.cuda.synchronize()
    for rnd in range(int(os.environ.get("ROUNDS", "4"))):
        for var in VARIANTS:
            lw, sp = var[0], var[1]
            sb.tune_set("gemm.loaders", lw)
            sb.tune_set("gemm.dma_spread", sp)
            sb.tune_set("gemm.dma_nt", var[2] if len(var) > 2 else 0)
            step()
            torch.cuda.synchronize()
            sb.timings_enable(True)
            sb.timings_filter("gemm")
            sb.timings_reset()
            for _ in range(10):
                step()
            torch.cuda.synchronize()
            ms, calls = sb.timings_get("gemm")
            sb.timings_enable(False)
            times[var].append(ms / calls)
            if ref is None:
                ref = vr.clone()
            elif not torch.equal(ref, vr):
                print(json.dumps({"error": "results differ", "lw": lw, "sp": sp,
                                  "maxdiff": float((ref - vr).abs().max())}), flush=True)
    sb.tune_set("gemm.loaders", 8)
    sb.tune_set("gemm.dma_spread", 1)
    sb.tune_set("gemm.dma_nt", 0)
    for var, t in times.items():
        t = sorted(t)
        print(json.dumps({"loaders": var[0], "spread": var[1], "nt": var[2] if len(var) > 2 else 0,
                          "gemm_ms_min": round(t[0], 4),
                          "gemm_ms_median": round(t[len(t) // 2], 4),
                          "TFLOPs_median": round(flops / t[len(t) // 2] / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
