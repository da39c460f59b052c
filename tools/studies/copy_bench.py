#!/usr/bin/env python3
"""Copy-kernel microbenchmark (not part of the product): per-call GB/s of
  (a) torch's contiguous device copy (reference point for "a memcpy of this size"),
  (b) the library's contiguous copy (identical labels),
  (c) the config-2p permute slice xyztsc -> tnsxyzc[n],
each replayed 64x inside a HIP graph so launch overhead is excluded.  Sizes: one 16^4 slice
(25 MB moved) and the whole 64-slice tensor (1.6 GB moved)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def graph_time(fn, reps=64, iters=3):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 1e3 / (reps * iters)


def main():
    dev = torch.device("cuda:0")
    L, n = 16, 64
    d0 = [L, L, L, L, 4, 3]
    d1 = [L, n, 4, L, L, L, 3]
    v0 = 1
    for x in d0:
        v0 *= x
    a = torch.randn(v0, dtype=torch.complex128, device=dev)
    b = torch.empty(v0, dtype=torch.complex128, device=dev)
    big = torch.empty(v0 * n, dtype=torch.complex128, device=dev)
    bigb = torch.empty_like(big)
    res = {}
    t = graph_time(lambda: b.copy_(a))
    res["torch_copy_25MB_GBps"] = 32 * v0 / t / 1e9
    p0 = [([0] * 6, d0)]
    t = graph_time(lambda: sb.copy(1.0, p0, "xyztsc", [0] * 6, d0, d0, [a], p0, "xyztsc",
                                   [0] * 6, d0, [b]))
    res["sbx_contig_25MB_GBps"] = 32 * v0 / t / 1e9
    p1 = [([0] * 7, d1)]
    t = graph_time(lambda: sb.copy(1.0, p0, "xyztsc", [0] * 6, d0, d0, [a], p1, "tnsxyzc",
                                   [0, 5, 0, 0, 0, 0, 0], d1, [big]))
    res["sbx_permute_slice_GBps"] = 32 * v0 / t / 1e9
    res["sbx_permute_slice_us"] = t * 1e6
    t = graph_time(lambda: bigb.copy_(big), reps=4)
    res["torch_copy_1.6GB_GBps"] = 32 * v0 * n / t / 1e9
    dd = [L, L, L, L, n, 4, 3]
    pd = [([0] * 7, dd)]
    pb = [([0] * 7, d1)]
    t = graph_time(lambda: sb.copy(1.0, pd, "xyztnsc", [0] * 7, dd, dd, [big], pb, "tnsxyzc",
                                   [0] * 7, d1, [bigb]), reps=4)
    res["sbx_permute_1.6GB_GBps"] = 32 * v0 * n / t / 1e9
    print(json.dumps({k: round(v, 1) for k, v in res.items()}))


if __name__ == "__main__":
    main()
