#!/usr/bin/env python3
"""Per-workgroup time line of the 3x3 lattice BSR kernels (config 3 shape, 16^4,
complex<double>; tools only): sbx_tune_set("bsr.probe", buffer) makes workgroup thread 0 store
its start / end (100 MHz real time) and its phases' shader-clock cycles.  Prints, per kernel
(chunked ELL9 with bsr.tile 0, tiled with bsr.tile 1) and n: the kernel span, workgroup
lifetime, workgroups resident per CU on average, and the mean cycles per phase
(tiled: issue = ids and entries, direct gathers issued; stage = LDS-DMA of values and staged x
until landed; sync = barrier wait; compute = products + y stores.  chunked: stage, compute)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import superbblas_amd as sb  # noqa: E402
from bsr_probe import columns  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    L = 16
    V = L ** 4
    jj = columns(os.environ.get("STENCIL", "stencil"), L)
    sb.tune_set("bsr.tile", 1)  # build the tile plan
    dim = [L, L, L, L, 1, 3]
    full = [([0] * 6, dim)]
    vals = torch.randn(V * 81, dtype=torch.complex128, device=dev)
    op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                       [torch.full((V,), 9, dtype=torch.int32, device=dev)],
                       [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])
    probe = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
    sb.tune_set("bsr.tile_min_cols", 1)
    sb.tune_set("bsr.tile_max_cols", 1 << 20)
    for tile in (0, 1):
        sb.tune_set("bsr.tile", tile)
        for ncols in [int(c) for c in os.environ.get("NCOLS", "1,12,64").split(",")]:
            dimx = [1, L, L, L, L, 1, 3, ncols]
            x = torch.randn(V * 3 * ncols, dtype=torch.complex128, device=dev)
            y = torch.empty_like(x)
            px = [([0] * 8, dimx)]

            def run():
                sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx,
                              [x], 0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            probe.zero_()
            sb.tune_set("bsr.probe", probe.data_ptr())
            run()
            torch.cuda.synchronize()
            sb.tune_set("bsr.probe", 0)
            p = probe.view(-1, 8).cpu().numpy()
            p = p[p[:, 0] != 0]
            start, end = p[:, 0], p[:, 1]
            span = (end.max() - start.min()) * 10.0  # ns
            life = (end - start) * 10.0
            out = {"kernel": "tiled" if tile else "chunked", "n": ncols, "workgroups": len(p),
                   "span_us": round(span / 1e3, 2),
                   "life_us_mean": round(life.mean() / 1e3, 3),
                   "life_us_p50": round(float(np.median(life)) / 1e3, 3),
                   "life_us_p90": round(float(np.percentile(life, 90)) / 1e3, 3),
                   "resident_per_cu": round(life.sum() / span / 256, 2),
                   "first_end_us": round((end.min() - start.min()) * 10.0 / 1e3, 2),
                   "last_start_us": round((start.max() - start.min()) * 10.0 / 1e3, 2)}
            names = ["issue", "stage", "sync", "compute"] if tile else [None, "stage", None, "compute"]
            for k, nm in zip(range(2, 6), names):
                if nm:
                    out["cyc_" + nm] = round(float(p[:, k].mean()), 0)
            print(json.dumps(out), flush=True)
    sb.tune_set("bsr.tile", 0)
    op.destroy()


if __name__ == "__main__":
    main()
