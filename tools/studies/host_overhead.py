"""Host-side cost per API call (Python wrapper + C++ planner + launch), on tiny tensors."""
import sys
import time

import torch

sys.path.insert(0, ".")
import superbblas_amd as sb  # noqa: E402

dev = torch.device("cuda:0")
d = [4, 4]
a = torch.ones(16, dtype=torch.complex128, device=dev)
b = torch.zeros(16, dtype=torch.complex128, device=dev)
p = [([0, 0], d)]
for _ in range(10):
    sb.copy(1.0, p, "xy", [0, 0], d, d, [a], p, "yx", [0, 0], d, [b])
torch.cuda.synchronize()
n = 2000
t = time.perf_counter()
for _ in range(n):
    sb.copy(1.0, p, "xy", [0, 0], d, d, [a], p, "yx", [0, 0], d, [b])
t = time.perf_counter() - t
torch.cuda.synchronize()
print("copy: %.2f us/call (host)" % (t / n * 1e6))
c = torch.zeros(16, dtype=torch.complex128, device=dev)
for _ in range(10):
    sb.contraction(1.0, p, [0, 0], d, d, "xy", False, [a], p, [0, 0], d, d, "zy", False, [b], 0.0,
                   p, [0, 0], d, d, "xz", [c])
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(n):
    sb.contraction(1.0, p, [0, 0], d, d, "xy", False, [a], p, [0, 0], d, d, "zy", False, [b], 0.0,
                   p, [0, 0], d, d, "xz", [c])
t = time.perf_counter() - t
torch.cuda.synchronize()
print("contraction: %.2f us/call (host)" % (t / n * 1e6))
s = sb.stream(0)
t = time.perf_counter()
for _ in range(n):
    torch.cuda.current_stream(0).cuda_stream
t = time.perf_counter() - t
print("torch.cuda.current_stream: %.2f us/call" % (t / n * 1e6))
