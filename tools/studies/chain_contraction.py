#!/usr/bin/env python3
"""The configs[4] chain's contraction alone (16^3 x 64 sites, complex<float>, n = 12:
pXYZTSCn (conj) x pXYZTsCN -> TSnsN, a batched GEMM with m = n = 48, k = 12 288, batch 64) by
GEMM tile shape (sbx_tune_set "gemm.t48": 0 = 64x64 tiles, 1..4 = the round-2 48x48 forms, 5 =
the library's choice, 6 = k-group workgroups, 13 / 14 / 16 = wave rings of 4 waves 8-deep, 4 waves
16-deep, 16 waves 8-deep; the default is 8 waves 8-deep); results
compared with torch.einsum.  Not part of the product."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    Ls, Lt, s_, c_, n = 16, 64, 4, 3, 12
    Lz = int(os.environ.get("LZ", Ls))  # (LZ: a shorter z extent, i.e. a shorter k, for the
    dx = [1, Ls, Ls, Lz, Lt, s_, c_, n]  # fixed-cost / per-k split of the launch time)
    V3 = Ls * Ls * Lz
    y = torch.randn(V3 * Lt * s_ * c_ * n, dtype=torch.complex64, device=dev)
    # DATA=zero / int: operands that switch fewer MFMA bits (a power / clock diagnostic)
    data = os.environ.get("DATA", "rand")
    if data == "zero":
        y.zero_()
    elif data == "int":
        y = torch.complex(torch.randint(-2, 3, y.shape, device=dev).float(),
                          torch.randint(-2, 3, y.shape, device=dev).float())
    dr = [Lt, s_, n, s_, n]
    vr = torch.empty(Lt * s_ * n * s_ * n, dtype=torch.complex64, device=dev)
    p_x, p_r = [([0] * 8, dx)], [([0] * 5, dr)]
    yv = y.view(V3, Lt, s_, c_, n)
    ref = torch.einsum("XTSCn,XTsCN->TSnsN", yv.conj(), yv).reshape(-1)
    fl = 8.0 * vr.numel() * V3 * c_
    combos = [(int(v), 1) for v in os.environ.get("T48", "0,1,2,3,4").split(",")]
    if os.environ.get("SHARE"):  # one slab image for both operands (the same memory) on / off
        combos = [(4, int(v)) for v in os.environ["SHARE"].split(",")] * 2
    splits = [int(v) for v in os.environ.get("SPLITS", "0").split(",")]  # 0: the library's choice
    combos = [(t, sh, sp) for t, sh in combos for sp in splits]
    for t48, share, nsplit in combos:
        sb.tune_set("gemm.t48", t48)
        sb.tune_set("gemm.share_ab", share)
        sb.tune_set("gemm.splits", nsplit)

        def f():
            sb.contraction(1.0, p_x, [0] * 8, dx, dx, "pXYZTSCn", True, [y], p_x, [0] * 8, dx, dx,
                           "pXYZTsCN", False, [y], 0.0, p_r, [0] * 5, dr, dr, "TSnsN", [vr])
        for _ in range(int(os.environ.get("WARM", "1"))):  # (WARM: clocks up before timing)
            f()
        torch.cuda.synchronize()
        err = (torch.linalg.vector_norm(vr - ref) / max(torch.linalg.vector_norm(ref), 1e-30)).item()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            f()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / 10 / 1e3
        print(json.dumps({"k": V3 * c_, "data": data, "t48": t48, "share_ab": share, "splits": nsplit, "ms": round(t * 1e3, 4),
                          "TFLOPs": round(fl / t / 1e12, 2),
                          "rel_err_vs_einsum": err}), flush=True)
    sb.tune_set("gemm.t48", 5)
    sb.tune_set("gemm.share_ab", 1)
    sb.tune_set("gemm.splits", 0)


if __name__ == "__main__":
    main()
