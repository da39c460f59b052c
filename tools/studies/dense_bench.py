#!/usr/bin/env python3
"""The dense batched solvers on the batches lattice codes give them: one small
matrix per lattice site (16^4 sites, 12x12 spin-color blocks, complex<double>: the clover-term
inverse) and the chain's 2-point matrices (64 time slices of 48x48, complex<float>).  Per case:
library time of the whole call (copy into the working layout, the kernel, copy back) and of the
kernel alone (library timers, median of 3 rounds of 10 calls), and the kernel's bytes (the
matrices in and out once) / time.  CASES=site12,t48; WAVE=1,0: the dense.wave settings (a wave
per matrix up to 16 x 16, or a workgroup per matrix).  Not part of the product."""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def hpd(nb, n, dt, dev):
    a = torch.randn(nb, n, n, dtype=dt, device=dev)
    return (a @ a.conj().transpose(1, 2) + n * torch.eye(n, dtype=dt, device=dev)).contiguous()


def timed(f, reps=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    out = []
    for _ in range(3):
        sb.timings_enable(True)
        sb.timings_reset()
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        ms, calls = sb.timings_get("dense")
        sb.timings_enable(False)
        out.append((wall, ms / max(calls, 1) / 1e3))
    return statistics.median(w for w, _ in out), statistics.median(k for _, k in out)


def wall_us(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    out = []
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) / reps * 1e6)
    return round(statistics.median(out), 1)


def overhead(dev):
    """OVERHEAD=1: where the inversion call's time beyond the kernel goes (site12, in place):
    the refill copy alone, the call alone (timers off), the call on a tiny batch (host + launch +
    the info check's round trip), and the kernel by the library timer"""
    nb, n, dt = 16 ** 4, 12, torch.complex128
    a0 = hpd(nb, n, dt, dev).reshape(-1)
    v = a0.clone()
    dim, full = [nb, n, n], [([0, 0, 0], [nb, n, n])]
    s0 = hpd(64, n, dt, dev).reshape(-1)
    small = s0.clone()
    ds, fs = [64, n, n], [([0, 0, 0], [64, n, n])]
    for op in ("inversion", "cholesky"):
        r = {"op": op,
             "refill_copy_us": wall_us(lambda: v.copy_(a0)),
             # (in place again on its own output: an inverse of the inverse; a Cholesky factor is
             # not a positive definite matrix, so Cholesky is timed with the refill only)
             "call_only_us": (wall_us(lambda: sb.inversion(full, dim, "tij", [v], "i", "j"))
                              if op == "inversion" else None),
             "call_64_matrices_us": wall_us(lambda: (small.copy_(s0), getattr(sb, op)(fs, ds, "tij", [small], "i", "j"))),
             "call_with_refill_us": wall_us(lambda: (v.copy_(a0), getattr(sb, op)(full, dim, "tij", [v], "i", "j")))}
        _, kern = timed(lambda: (v.copy_(a0), getattr(sb, op)(full, dim, "tij", [v], "i", "j")))
        r["kernel_us"] = round(kern * 1e6, 1)
        print(json.dumps(r), flush=True)


def main():
    dev = torch.device("cuda:0")
    if os.environ.get("OVERHEAD"):
        return overhead(dev)
    cases = os.environ.get("CASES", "site12,t48").split(",")
    shapes = {"site12": (16 ** 4, 12, torch.complex128), "t48": (64, 48, torch.complex64),
              "site3": (16 ** 4, 3, torch.complex128)}
    for name in cases:
        nb, n, dt = shapes[name]
        es = torch.empty(0, dtype=dt).element_size()
        dim = [nb, n, n]
        full = [([0, 0, 0], dim)]
        a0 = hpd(nb, n, dt, dev)
        for op, wv in [(op, wv) for op in ("cholesky", "inversion")
                       for wv in [int(x) for x in os.environ.get("WAVE", "1,0").split(",")]]:
            sb.tune_set("dense.wave", wv)
            v = a0.clone().reshape(-1)

            def f():
                v.copy_(a0.reshape(-1))
                getattr(sb, op)(full, dim, "tij", [v], "i", "j")
            wall, kern = timed(f)
            by = 2.0 * nb * n * n * es
            print(json.dumps({"case": name, "op": op, "wave": wv, "matrices": nb, "n": n, "dtype": str(dt),
                              "call_us": round(wall * 1e6, 1), "kernel_us": round(kern * 1e6, 1),
                              "kernel_GBps": round(by / kern / 1e9, 1)}), flush=True)
        # solves with the factor / the matrix: x with C's column labels, 12 right-hand sides
        nr = 12
        u = a0.clone().reshape(-1)
        sb.cholesky(full, dim, "tij", [u], "i", "j")
        dimx = [nb, n, nr]
        px = [([0, 0, 0], dimx)]
        x = torch.randn(nb * n * nr, dtype=dt, device=dev)
        y = torch.empty_like(x)
        for op, mat, wv in [(op, mat, wv) for op, mat in (("trsm", u), ("gesm", a0.reshape(-1)))
                            for wv in [int(x) for x in os.environ.get("WAVE", "1,0").split(",")]]:
            sb.tune_set("dense.wave", wv)

            def f():
                getattr(sb, op)(1.0, full, dim, "tij", [mat], "i", "j", px, dimx, "tjr", [x], px,
                                dimx, "tir", [y])
            wall, kern = timed(f)
            by = 16.0 * nb * n * n * es / 16 + 2.0 * nb * n * nr * es
            print(json.dumps({"case": name, "op": op, "wave": wv, "matrices": nb, "n": n, "rhs": nr,
                              "dtype": str(dt), "call_us": round(wall * 1e6, 1),
                              "kernel_us": round(kern * 1e6, 1),
                              "kernel_GBps": round(by / kern / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
