#!/usr/bin/env python3
"""Tile-shape sweep of the config-2p permute (not part of the product): the bench's 64-slice
xyztsc -> tnsxyzc[n] loop (complex<double>) replayed as a HIP graph, for several copy kernel
shapes set through sbx_tune_set; torch's contiguous copy into the same 64 distinct slices is the
memcpy reference for this access pattern."""
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


def graph_time(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 1e3 / iters


def main():
    dev = torch.device("cuda:0")
    L, n = 16, 64
    d0 = [L, L, L, L, 4, 3]
    d1 = [L, n, 4, L, L, L, 3]
    a = torch.randn(vol(d0), dtype=torch.complex128, device=dev)
    af = a.to(torch.complex64)
    b = torch.zeros(vol(d1), dtype=torch.complex128, device=dev)
    p0, p1 = [([0] * 6, d0)], [([0] * 7, d1)]
    by = 32.0 * vol(d1)
    bv = b.view(n, -1)  # contiguous slices of the same sizes (memcpy reference)

    def torch_slices():
        for k in range(n):
            bv[k].copy_(a)
    t = graph_time(torch_slices)
    print(json.dumps({"case": "torch contiguous copy x64 slices", "GBps": round(by / t / 1e9, 1),
                      "us_per_slice": round(t / n * 1e6, 2)}), flush=True)
    # reference: torch's permute of the same slices
    ref = b.clone()
    rv = ref.view(L, n, 4, L, L, L, 3)
    src = a.view(L, L, L, L, 4, 3).permute(3, 4, 0, 1, 2, 5)  # xyztsc -> tsxyzc
    for k in range(n):
        rv[:, k].copy_(src)
    configs = [dict(), dict(budget=1536), dict(budget=512), dict(nt=-1)]
    if os.environ.get("PERMUTE_CONFIGS"):
        configs = json.loads(os.environ["PERMUTE_CONFIGS"])
    defaults = {"budget": 0, "run": 0, "nt": 0, "trans": 0}
    for cfg in configs:
        for k, v in defaults.items():
            sb.tune_set("copy." + k, cfg.get(k, v))
        b.zero_()

        def run():
            for k in range(n):
                sb.copy(1.0, p0, "xyztsc", [0] * 6, d0, d0, [a], p1, "tnsxyzc",
                        [0, k, 0, 0, 0, 0, 0], d1, [b])
        t = graph_time(run)
        torch.cuda.synchronize()
        ok = bool(torch.equal(b, ref))

        def run_f():
            for k in range(n):
                sb.copy(1.0, p0, "xyztsc", [0] * 6, d0, d0, [af], p1, "tnsxyzc",
                        [0, k, 0, 0, 0, 0, 0], d1, [b])
        t2 = graph_time(run_f)
        torch.cuda.synchronize()
        ok_f = bool(torch.equal(b, ref.to(torch.complex64).to(torch.complex128)))
        bf = torch.zeros(vol(d1), dtype=torch.complex64, device=dev)

        def run_ff():
            for k in range(n):
                sb.copy(1.0, p0, "xyztsc", [0] * 6, d0, d0, [af], p1, "tnsxyzc",
                        [0, k, 0, 0, 0, 0, 0], d1, [bf])
        t3 = graph_time(run_ff)
        torch.cuda.synchronize()
        ok_ff = bool(torch.equal(bf, ref.to(torch.complex64)))
        print(json.dumps({"case": cfg, "GBps": round(by / t / 1e9, 1),
                          "us_per_slice": round(t / n * 1e6, 2), "exact": ok,
                          "cf2cd_GBps": round(24.0 * vol(d1) / t2 / 1e9, 1), "cf2cd_exact": ok_f,
                          "cf2cf_GBps": round(16.0 * vol(d1) / t3 / 1e9, 1), "cf2cf_exact": ok_ff}),
              flush=True)


    for k, v in defaults.items():
        sb.tune_set("copy." + k, v)


if __name__ == "__main__":
    main()
