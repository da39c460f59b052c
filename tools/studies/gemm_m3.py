#!/usr/bin/env python3
"""Complex GEMM in the 4-multiplication vs the 3-multiplication (Gauss) form (not part of the
product; sbx_tune_set("gemm.m3")): the config-2 lattice contraction (complex<double>, 16^4,
n = 64) and the chain's contraction (complex<float>, 16^3 x 64, T S n s N), GEMM kernel time from
the library timers and the relative difference of the two results."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def vol(d):
    n = 1
    for x in d:
        n *= x
    return n


def timed(f, reps=10):
    f()
    torch.cuda.synchronize()
    sb.timings_enable(True)
    sb.timings_reset()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    ms, calls = sb.timings_get("gemm")
    rms, rcalls = sb.timings_get("gemm_splitk_reduce")
    sb.timings_enable(False)
    return ms / max(calls, 1), rms / max(rcalls, 1)


def main():
    dev = torch.device("cuda:0")
    # config 2
    L, n = 16, 64
    d0 = [L, n, 4, L, L, L, 3]
    dr = [L, n, 4, n, 4]
    v0 = torch.randn(vol(d0), dtype=torch.complex128, device=dev)
    v1 = torch.randn(vol(d0), dtype=torch.complex128, device=dev)
    z7, z5 = [0] * 7, [0] * 5
    flops = 8.0 * L * (L ** 3 * 3) * (n * 4) ** 2
    res = {}
    for m3 in (-1, 1):
        sb.tune_set("gemm.m3", m3)
        vr = torch.zeros(vol(dr), dtype=torch.complex128, device=dev)

        def f():
            sb.contraction(1.0, [(z7, d0)], z7, d0, d0, "tnsxyzc", False, [v0], [(z7, d0)], z7,
                           d0, d0, "tNSxyzc", False, [v1], 0.0, [(z5, dr)], z5, dr, dr, "tNSns",
                           [vr])
        ms, rms = timed(f)
        res[m3] = vr.clone()
        print(json.dumps({"case": "config2 cdouble", "m3": m3, "gemm_ms": round(ms, 4),
                          "reduce_ms": round(rms, 4), "TFLOPs": round(flops / ms / 1e9, 2)}),
              flush=True)
    err = float((res[-1] - res[1]).abs().max() / res[-1].abs().max())
    print(json.dumps({"case": "config2 cdouble", "max_rel_diff_m3_vs_m4": err}), flush=True)
    # the chain's contraction (complex<float>)
    Ls, Lt, nc = 16, 64, 12
    dx = [1, Ls, Ls, Ls, Lt, 4, 3, nc]
    y = torch.randn(vol(dx), dtype=torch.complex64, device=dev)
    drr = [Lt, 4, nc, 4, nc]
    px, pr = [([0] * 8, dx)], [([0] * 5, drr)]
    flops = 8.0 * Lt * (Ls ** 3 * 3) * (4 * nc) ** 2
    res = {}
    for m3 in (-1, 1):
        sb.tune_set("gemm.m3", m3)
        vr = torch.zeros(vol(drr), dtype=torch.complex64, device=dev)

        def g():
            sb.contraction(1.0, px, [0] * 8, dx, dx, "pXYZTSCn", True, [y], px, [0] * 8, dx, dx,
                           "pXYZTsCN", False, [y], 0.0, pr, [0] * 5, drr, drr, "TSnsN", [vr])
        ms, rms = timed(g)
        res[m3] = vr.clone()
        print(json.dumps({"case": "chain cfloat", "m3": m3, "gemm_ms": round(ms, 4),
                          "reduce_ms": round(rms, 4), "TFLOPs": round(flops / ms / 1e9, 2)}),
              flush=True)
    err = float((res[-1] - res[1]).abs().max() / res[-1].abs().max())
    print(json.dumps({"case": "chain cfloat", "max_rel_diff_m3_vs_m4": err}), flush=True)
    sb.tune_set("gemm.m3", 0)


if __name__ == "__main__":
    main()
