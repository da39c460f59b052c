#!/usr/bin/env python3
"""Config-2 contraction (16^4, n = 64, complex<double>) by split-K factor (sbx_tune_set
"gemm.splits"; 0 = the library's choice), warm round robin; not part of the product."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    L, n = 16, 64
    d0 = [L, n, 4, L, L, L, 3]
    dr = [L, n, 4, n, 4]
    v0 = torch.randn(L * n * 4 * L ** 3 * 3, dtype=torch.complex128, device=dev)
    v1 = torch.randn_like(v0)
    vr = torch.zeros(L * n * 4 * n * 4, dtype=torch.complex128, device=dev)
    z7, z5 = [0] * 7, [0] * 5

    def step():
        sb.contraction(1.0, [(z7, d0)], z7, d0, d0, "tnsxyzc", False, [v0], [(z7, d0)], z7, d0,
                       d0, "tNSxyzc", False, [v1], 0.0, [(z5, dr)], z5, dr, dr, "tNSns", [vr])
    t0 = time.time()
    while time.time() - t0 < 1.0:
        step()
    torch.cuda.synchronize()
    splits = [int(v) for v in os.environ.get("SPLITS", "0,2,3,4,5,6,8").split(",")]
    res = {s: [] for s in splits}
    ref = None
    for _ in range(3):
        for sp in splits:
            sb.tune_set("gemm.splits", sp)
            step()
            torch.cuda.synchronize()
            if ref is None:
                ref = vr.clone()
            err = float((vr - ref).abs().max() / ref.abs().max())
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                step()
            e.record()
            torch.cuda.synchronize()
            res[sp].append((s.elapsed_time(e) / 20, err))
    sb.tune_set("gemm.splits", 0)
    for sp in splits:
        print(json.dumps({"splits": sp, "ms_min": round(min(t for t, _ in res[sp]), 4),
                          "ms": [round(t, 4) for t, _ in res[sp]],
                          "rel_diff_vs_first": max(e for _, e in res[sp])}), flush=True)


if __name__ == "__main__":
    main()
