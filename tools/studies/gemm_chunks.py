#!/usr/bin/env python3
"""GEMM time of the config-2 contraction issued whole vs as 4 T-chunks (not part of the
product): the N > 1 bench pipelines the cross-rank reduction behind T-chunked GEMMs
(contraction.cpp, 3+4 pipelined); this measures what the chunking costs on one GPU."""
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


def main():
    dev = torch.device("cuda:0")
    L, n = 16, 64
    d0 = [L, n, 4, L, L, L, 3]
    dr = [L, n, 4, n, 4]
    v0 = torch.randn(vol(d0), dtype=torch.complex128, device=dev)
    v1 = torch.randn(vol(d0), dtype=torch.complex128, device=dev)
    vr = torch.zeros(vol(dr), dtype=torch.complex128, device=dev)
    z7, z5 = [0] * 7, [0] * 5
    for nch, splits in ((1, 0), (2, 0), (4, 0), (1, 4), (1, 8), (1, 16)):
        sb.tune_set("gemm.splits", splits)
        tl = L // nch

        def f():
            for c in range(nch):
                f0 = [c * tl] + [0] * 6
                s0 = [tl] + d0[1:]
                fr = [c * tl] + [0] * 4
                sr = [tl] + dr[1:]
                sb.contraction(1.0, [(z7, d0)], f0, s0, d0, "tnsxyzc", False, [v0], [(z7, d0)],
                               f0, s0, d0, "tNSxyzc", False, [v1], 0.0, [(z5, dr)], fr, sr, dr,
                               "tNSns", [vr])
        f()
        torch.cuda.synchronize()
        sb.timings_enable(True)
        sb.timings_reset()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            f()
        e.record()
        torch.cuda.synchronize()
        ms, calls = sb.timings_get("gemm")
        rms, _ = sb.timings_get("gemm_splitk_reduce")
        sb.timings_enable(False)
        print(json.dumps({"chunks": nch, "splits": splits, "step_ms": round(s.elapsed_time(e) / 10, 4),
                          "gemm_ms_per_step": round(ms / 10, 4),
                          "reduce_ms_per_step": round(rms / 10, 4)}), flush=True)


if __name__ == "__main__":
    main()
