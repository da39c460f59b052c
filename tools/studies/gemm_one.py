#!/usr/bin/env python3
"""The config-2 GEMM alone, REPS times (for rocprofv3 counter passes; not part of the product).
Env: LOADERS / SPREAD (gemm.loaders / gemm.dma_spread), REPS."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402

dev = torch.device("cuda:0")
L, n = 16, 64
d0 = [L, n, 4, L, L, L, 3]
dr = [L, n, 4, n, 4]
vol0 = L * n * 4 * L * L * L * 3
g = torch.Generator(device=dev).manual_seed(5)
v0 = torch.randn(vol0, dtype=torch.complex128, device=dev, generator=g)
v1 = torch.randn(vol0, dtype=torch.complex128, device=dev, generator=g)
vr = torch.zeros(L * n * 4 * n * 4, dtype=torch.complex128, device=dev)
z7, z5 = [0] * 7, [0] * 5
sb.tune_set("gemm.loaders", int(os.environ.get("LOADERS", "0")))
sb.tune_set("gemm.dma_spread", int(os.environ.get("SPREAD", "1")))
for _ in range(int(os.environ.get("REPS", "20"))):
    sb.contraction(1.0, [(z7, d0)], z7, d0, d0, "tnsxyzc", False, [v0], [(z7, d0)], z7, d0, d0,
                   "tNSxyzc", False, [v1], 0.0, [(z5, dr)], z5, dr, dr, "tNSns", [vr])
torch.cuda.synchronize()
