#!/usr/bin/env python3
"""Host time per copy() call of the Python mirror (ctypes) on the config-2p slice loop, with a
cProfile breakdown; not part of the product (the C ABI's own cost: tools/capi_overhead)."""
import time, torch, cProfile, pstats, sys, os
sys.path.insert(0, os.getcwd())
import superbblas_amd as sb
dev = torch.device("cuda:0")
L, n = 16, 64
d0 = [L, L, L, L, 4, 3]; d1 = [L, n, 4, L, L, L, 3]
a = torch.randn(L**4*12, dtype=torch.complex128, device=dev)
b = torch.zeros(L**4*12*n, dtype=torch.complex128, device=dev)
p0, p1 = [([0]*6, d0)], [([0]*7, d1)]
def loop():
    for k in range(n):
        sb.copy(1.0, p0, "xyztsc", [0]*6, d0, d0, [a], p1, "tnsxyzc", [0, k, 0, 0, 0, 0, 0], d1, [b])
loop(); torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20): loop()
host = (time.perf_counter() - t) / 20 / n
torch.cuda.synchronize()
print("host us per copy", host * 1e6)
pr = cProfile.Profile(); pr.enable()
for _ in range(20): loop()
pr.disable(); torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(12)
