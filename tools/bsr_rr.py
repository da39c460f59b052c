#!/usr/bin/env python3
"""Round-robin A/B timing of the 9-point 3x3 BSR kernel forms on a warm GPU (config 3, 16^4,
complex<double>, x and y row major; not part of the product).  Each configuration is a set of
sbx_tune_set keys; the GPU is brought to clock first (0.5 s of the kernel), then every
configuration is timed in turn, ROUNDS times (min and median), so clock drift does not favour
the configurations timed last.  Outputs are checked against the first configuration's."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import superbblas_amd as sb  # noqa: E402
from bsr_split_sweep import lattice_op  # noqa: E402

CONFIGS = {
    "chunked": {"bsr.split_max_cols": 0, "bsr.ell9_ilv": 1},
    "chunked_ilv2": {"bsr.split_max_cols": 0, "bsr.ell9_ilv": 2},
    "split_cw1_jb3": {"bsr.split_cw": 1, "bsr.split_jb": 3, "bsr.split_ilv": 1},
    "split_cw2_jb3": {"bsr.split_cw": 2, "bsr.split_jb": 3, "bsr.split_ilv": 1},
    "split_cw2_jb3_ilv2": {"bsr.split_cw": 2, "bsr.split_jb": 3, "bsr.split_ilv": 2},
    "split_cw2_jb9_ilv2": {"bsr.split_cw": 2, "bsr.split_jb": 9, "bsr.split_ilv": 2},
    "cw2_jb3_sep": {"bsr.split_cw": 2, "bsr.split_jb": 3, "bsr.split_ovl": 0},
    "cw2_jb3_ovl": {"bsr.split_cw": 2, "bsr.split_jb": 3, "bsr.split_ovl": 1},
    "cw1_jb3_ovl": {"bsr.split_cw": 1, "bsr.split_jb": 3, "bsr.split_ovl": 1},
    "cw2_jb3_ovl_nt512": {"bsr.split_cw": 2, "bsr.split_jb": 3, "bsr.split_ovl": 1, "bsr.split_nt": 512},
    "cw1_jb3_ovl_nt512": {"bsr.split_cw": 1, "bsr.split_jb": 3, "bsr.split_ovl": 1, "bsr.split_nt": 512},
    "cw2_jb1_ovl": {"bsr.split_cw": 2, "bsr.split_jb": 1, "bsr.split_ovl": 1},
    "ilv1": {"bsr.split_ilv": 1}, "ilv4": {"bsr.split_ilv": 4}, "ilv8": {"bsr.split_ilv": 8},
    "rw10": {"bsr.split_rw": 10}, "rw11": {"bsr.split_rw": 11}, "rw12": {"bsr.split_rw": 12},
    "rw13": {"bsr.split_rw": 13}, "rw14": {"bsr.split_rw": 14},
    "default": {},
}
BASE = {"bsr.split_max_cols": 1 << 20, "bsr.row_max_cols": 0, "bsr.split_cw": 0,
        "bsr.split_jb": 0, "bsr.split_ilv": 2, "bsr.ell9_ilv": 2, "bsr.tile": 0,
        "bsr.split_ovl": 1, "bsr.split_nt": 0, "bsr.split_rw": 0}
DEFAULTS = {"bsr.split_max_cols": 32, "bsr.row_max_cols": 3, "bsr.split_cw": 0,
            "bsr.split_jb": 0, "bsr.split_ilv": 2, "bsr.ell9_ilv": 2, "bsr.tile": 0,
            "bsr.split_ovl": 1, "bsr.split_nt": 0, "bsr.split_rw": 0}


def main():
    dev = torch.device("cuda:0")
    L = 16
    V = L ** 4
    op = lattice_op(sb, dev, L)
    names = os.environ.get("CONFIGS", ",".join(CONFIGS)).split(",")
    for ncols in [int(c) for c in os.environ.get("NCOLS", "8,12,16,24,32,64").split(",")]:
        dimx = [1, L, L, L, L, 1, 3, ncols]
        x = torch.randn(V * 3 * ncols, dtype=torch.complex128, device=dev)
        y = torch.empty_like(x)
        px = [([0] * 8, dimx)]
        by = 16.0 * (81 * V + 2 * 3 * V * ncols) + 4.0 * (9 * V + V + 1)

        def run():
            sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx, [x],
                          0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])

        def apply(name):
            keys = dict(DEFAULTS) if name == "default" else dict(BASE)
            keys.update(CONFIGS[name])
            for k, v in keys.items():
                sb.tune_set(k, v)
        apply(names[0])
        t0 = time.time()
        while time.time() - t0 < 0.5:
            run()
            torch.cuda.synchronize()
        times = {n: [] for n in names}
        ref, err, kern = None, {}, {}
        for _ in range(int(os.environ.get("ROUNDS", "4"))):
            for name in names:
                apply(name)
                run()
                torch.cuda.synchronize()
                if ref is None:
                    ref = y.clone()
                err[name] = float((y - ref).abs().max() / ref.abs().max())
                kern[name] = sb.tune_get("bsr.last_kernel")
                sb.timings_enable(True)
                sb.timings_filter("bsr")
                sb.timings_reset()
                for _ in range(10):
                    run()
                torch.cuda.synchronize()
                ms, calls = sb.timings_get("bsr")
                sb.timings_enable(False)
                sb.timings_filter(None)
                times[name].append(ms / calls / 1e3)
        for name in names:
            t = min(times[name])
            print(json.dumps({"n": ncols, "config": name, "kernel_form": kern[name],
                              "kernel_us_min": round(t * 1e6, 2),
                              "kernel_us_median": round(float(np.median(times[name])) * 1e6, 2),
                              "frac_hbm": round(by / t / 8e12, 4), "rel_err": err[name]}),
                  flush=True)
        del x, y, ref
    for k, v in DEFAULTS.items():
        sb.tune_set(k, v)
    op.destroy()


if __name__ == "__main__":
    main()
