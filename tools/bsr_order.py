#!/usr/bin/env python3
"""Row-order experiment for the 3x3 lattice BSR (config 3, 16^4, complex<double>; not part of the
product): the same 9-point operator with its block rows (sites) listed in
  natural  -- lexicographic x, y, z, t (t fastest), the order of the bench operator;
  blocked  -- the lattice cut into 8 blocks of 8x8x8x16 (one per XCD: the kernel deals
              consecutive row chunks to one XCD), each block swept along t with its 8x8x8 plane
              fastest, so a site's 8 neighbours' x rows are touched within ~3 planes (~2 MB of
              L2 traffic) instead of 4096 sites apart.
Only the row order changes (y comes out permuted); the kernel time shows how much of the x
re-fetch traffic the order removes.  Prints one JSON line per (order, n)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import superbblas_amd as sb  # noqa: E402


def morton_key(c, bits):
    """interleave the bits of the 4 coordinates (t lowest)"""
    k = np.zeros(len(c), np.int64)
    for b in range(bits):
        for d in range(4):
            k |= ((c[:, d] >> b) & 1).astype(np.int64) << (4 * b + (3 - d))
    return k


def sites_in_order(L, order):
    idx = np.arange(L ** 4)
    nat = np.array(np.unravel_index(idx, (L, L, L, L))).T
    if order == "natural":
        return nat
    if order == "morton":
        return nat[np.argsort(morton_key(nat, int(np.log2(L))), kind="stable")]
    if order == "tile4":
        # XCD blocks of (L/2)^3 x L, inside: 4^4 tiles in Morton order, sites natural in a tile
        blk = (nat[:, 0] // (L // 2)) * 4 + (nat[:, 1] // (L // 2)) * 2 + nat[:, 2] // (L // 2)
        tile = nat // 4
        tkey = morton_key(tile, int(np.log2(L // 4)) + 1)
        inner = ((nat[:, 0] % 4 * 4 + nat[:, 1] % 4) * 4 + nat[:, 2] % 4) * 4 + nat[:, 3] % 4
        key = (blk.astype(np.int64) << 40) | (tkey << 8) | inner
        return nat[np.argsort(key, kind="stable")]
    if order.startswith("sim"):
        # "sim16-4-4-4": each XCD's rows (one eighth, consecutive) = one region of full c0 x halves
        # of c1, c2, c3, swept in blocks of 16 x 4 x 4 x 4 (the L2 LRU model's best order);
        # run with the XCD interleave off (bsr.ell9_ilv / bsr.split_ilv 1)
        import itertools
        bs = [int(v) for v in order[3:].split("-")]
        out = []
        h = L // 2
        for k in range(8):
            hh = [(k >> 2) & 1, (k >> 1) & 1, k & 1]
            lo, ext = [0, hh[0] * h, hh[1] * h, hh[2] * h], [L, h, h, h]
            nb = [ext[d] // bs[d] for d in range(4)]
            for B in itertools.product(*[range(v) for v in nb]):
                for a in itertools.product(*[range(v) for v in bs]):
                    out.append([lo[d] + B[d] * bs[d] + a[d] for d in range(4)])
        return np.array(out)
    h = L // 2
    out = []
    for bx in range(2):
        for by in range(2):
            for bz in range(2):
                t, x, y, z = np.meshgrid(np.arange(L), np.arange(h), np.arange(h), np.arange(h),
                                         indexing="ij")
                out.append(np.stack([x.ravel() + bx * h, y.ravel() + by * h, z.ravel() + bz * h,
                                     t.ravel()], 1))
    return np.concatenate(out)


def main():
    dev = torch.device("cuda:0")
    L = 16
    V = L ** 4
    for order in sys.argv[1:] or ("natural", "blocked", "morton", "tile4"):
        sites = sites_in_order(L, order)
        jj = np.zeros((V, 9, 6), np.int32)
        jj[:, 0, :4] = sites
        k = 1
        for d in range(4):
            for s in (-1, 1):
                c = sites.copy()
                c[:, d] = (c[:, d] + s) % L
                jj[:, k, :4] = c
                k += 1
        dim = [L, L, L, L, 1, 3]
        full = [([0] * 6, dim)]
        vals = torch.randn(V * 81, dtype=torch.complex128, device=dev)
        op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                           [torch.full((V,), 9, dtype=torch.int32, device=dev)],
                           [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])
        ilv = 1 if order.startswith("sim") else 2
        sb.tune_set("bsr.ell9_ilv", ilv)
        sb.tune_set("bsr.split_ilv", ilv)
        cases = [(12, 0), (64, 0)] if os.environ.get("ORDER_QUICK") else \
            [(1, 0), (12, 0), (64, 0)] + [(64, c) for c in (32, 16)] + [(12, 6)]
        for ncols, split in cases:
            sb.tune_set("bsr.colsplit", split)
            dimx = [1, L, L, L, L, 1, 3, ncols]
            x = torch.randn(V * 3 * ncols, dtype=torch.complex128, device=dev)
            y = torch.empty_like(x)
            px = [([0] * 8, dimx)]

            def run():
                sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx,
                              [x], 0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])
            run()
            torch.cuda.synchronize()
            sb.timings_enable(True)
            sb.timings_filter("bsr")
            sb.timings_reset()
            for _ in range(10):
                run()
            torch.cuda.synchronize()
            ms, calls = sb.timings_get("bsr")
            sb.timings_enable(False)
            sb.timings_filter(None)
            t = ms / 10 / 1e3  # one product = all its column passes
            by = 16.0 * (81 * V + 2 * 3 * V * ncols) + 4.0 * (9 * V + V + 1)
            print(json.dumps({"order": order, "ilv": ilv, "n": ncols, "colsplit": split,
                              "kernel_us": round(t * 1e6, 2),
                              "GBps": round(by / t / 1e9, 1),
                              "frac_hbm": round(by / t / 8e12, 4)}), flush=True)
        sb.tune_set("bsr.colsplit", 0)
        sb.tune_set("bsr.ell9_ilv", 2)
        sb.tune_set("bsr.split_ilv", 2)
        op.destroy()


if __name__ == "__main__":
    main()
