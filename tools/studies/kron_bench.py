#!/usr/bin/env python3
"""Kronecker BSR microbenchmark (not part of the product): 16^4 periodic 9-point Wilson-like
stencil, color 3x3 blocks per (site, direction) times a 4x4 spin matrix per direction
(1 -/+ gamma_mu in a chiral basis: two nonzeros per row; identity for the self term),
x pXYZTCnS -> y pxyztcns; kernel time from the library's HIP-event timers."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def wilson_spin_matrices(dense=False):
    """9 spin matrices: identity, then 1 - g_mu, 1 + g_mu for mu = x, y, z, t (chiral basis)."""
    i = 1j
    g = [np.array([[0, 0, 0, i], [0, 0, i, 0], [0, -i, 0, 0], [-i, 0, 0, 0]]),
         np.array([[0, 0, 0, -1], [0, 0, 1, 0], [0, 1, 0, 0], [-1, 0, 0, 0]]),
         np.array([[0, 0, i, 0], [0, 0, 0, -i], [-i, 0, 0, 0], [0, i, 0, 0]]),
         np.array([[0, 0, 1, 0], [0, 0, 0, 1], [1, 0, 0, 0], [0, 1, 0, 0]])]
    ks = [np.eye(4)]
    for gm in g:
        ks += [np.eye(4) - gm, np.eye(4) + gm]
    k = np.array(ks, np.complex128)
    if dense:
        k = k + 0.5
    return k.reshape(-1)


def lattice(L):
    V = L ** 4
    sites = np.array(np.unravel_index(np.arange(V), (L, L, L, L))).T
    jj = np.zeros((V, 9, 6), np.int32)
    jj[:, 0, :4] = sites
    k = 1
    for d in range(4):
        for s in (-1, 1):
            c = sites.copy()
            c[:, d] = (c[:, d] + s) % L
            jj[:, k, :4] = c
            k += 1
    return np.full(V, 9, np.int32), jj.reshape(-1)


def run(L, ncols, dev, dtype=torch.complex128, dense=False, reps=20):
    spin, color = 4, 3
    dim = [L, L, L, L, spin, color]
    V = L ** 4
    ii, jj = lattice(L)
    vals = torch.randn(V * 9 * color * color, dtype=dtype, device=dev)
    kron = torch.from_numpy(wilson_spin_matrices(dense)).to(dtype).to(dev)
    full = [([0] * 6, dim)]
    blk, kr = [1, 1, 1, 1, 1, color], [1, 1, 1, 1, spin, 1]
    op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, False,
                            [torch.from_numpy(ii).to(dev)], [torch.from_numpy(jj).to(dev)], [vals],
                            [kron])
    dimx = [1, L, L, L, L, color, ncols, spin]
    x = torch.randn(V * color * ncols * spin, dtype=dtype, device=dev)
    y = torch.empty_like(x)
    px = [([0] * 8, dimx)]

    def f():
        sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTCnS", [0] * 8, dimx, dimx, [x], 0.0,
                      px, "pxyztcns", [0] * 8, dimx, dimx, "p", [y])
    f()
    torch.cuda.synchronize()
    sb.timings_enable(True)
    sb.timings_reset()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    ms, calls = sb.timings_get("bsr")
    sb.timings_enable(False)
    op.destroy()
    t = ms / calls / 1e3
    es = x.element_size()
    # algorithmic bytes: color blocks, x and y once, the column indices
    by = es * (9 * 9 * V + 2 * 12 * V * ncols) + 4.0 * 9 * V
    # reference flop model (bsr.h:484-497, row major): (ki*b*b + kd*ki*b) per nonzero and rhs
    fl = 8.0 * (4 * 9 + 16 * 3) * 9 * V * ncols
    return {"dtype": str(dtype).split(".")[-1], "spin_matrices": "dense" if dense else "wilson",
            "n": ncols, "us": round(t * 1e6, 1), "GBps": round(by / t / 1e9, 1),
            "GFLOPs": round(fl / t / 1e9, 1)}


def main():
    dev = torch.device("cuda", 0)
    L = int(os.environ.get("L", "16"))
    only = os.environ.get("KRON_ONLY")  # e.g. "complex128:12"
    if os.environ.get("KRON_PACKS"):  # packed column slots of the MFMA kernel on / off, round robin
        for n in [int(v) for v in os.environ.get("KRON_NS", "8,12").split(",")]:
            for rnd in range(2):
                for pk in [int(v) for v in os.environ["KRON_PACKS"].split(",")]:
                    sb.tune_set("bsr.kron_pack", pk)
                    r = run(L, n, dev)
                    r.update({"kron_pack": pk, "round": rnd,
                              "kernel_form": sb.tune_get("bsr.last_kernel")})
                    print(json.dumps(r), flush=True)
        sb.tune_set("bsr.kron_pack", 1)
        return
    if only:
        dt, n = only.split(":")
        print(json.dumps(run(L, int(n), dev, getattr(torch, dt), False)), flush=True)
        return
    for dtype in (torch.complex128, torch.complex64):
        for dense in (False, True):
            for n in (1, 12, 24):
                print(json.dumps(run(L, n, dev, dtype, dense)), flush=True)


if __name__ == "__main__":
    main()
