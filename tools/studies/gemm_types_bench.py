#!/usr/bin/env python3
"""GEMM throughput per type (not part of the product): the lattice contraction's
('T','N') m = n = 256, k = 12288, batch 16 shape through sbx_xgemm_batch_strided for
complex<double>, double, complex<float>, float; kernel time from the library timers."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    m = n = 256
    k, batch = 12288, 16
    for dt, mult in ((torch.complex128, 8), (torch.float64, 2), (torch.complex64, 8),
                     (torch.float32, 2)):
        a = torch.randn(batch * m * k, dtype=dt, device=dev)
        b = torch.randn(batch * n * k, dtype=dt, device=dev)
        c = torch.empty(batch * m * n, dtype=dt, device=dev)

        def f():
            sb.xgemm_batch_strided("T", "N", m, n, k, 1.0, a, k, m * k, b, k, n * k, 0.0, c, m,
                                   m * n, batch)
        f()
        torch.cuda.synchronize()
        sb.timings_enable(True)
        sb.timings_reset()
        for _ in range(10):
            f()
        torch.cuda.synchronize()
        ms, calls = sb.timings_get("gemm")
        sb.timings_enable(False)
        t = ms / calls / 1e3
        ref = torch.einsum("bik,bjk->bji", a.view(batch, m, k), b.view(batch, n, k)).reshape(-1)
        err = (torch.linalg.vector_norm(c - ref) / torch.linalg.vector_norm(ref)).item()
        print(json.dumps({"dtype": str(dt), "ms": round(t * 1e3, 3),
                          "TFLOPs": round(mult * m * n * k * batch / t / 1e12, 2),
                          "rel_err": err}))


if __name__ == "__main__":
    main()
