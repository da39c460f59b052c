"""The configs[4] chain's distributed geometry (xyz grid, operator with a one-site halo domain) as
ONE process holding every rank's part as a component on its GPU: the same planner, copies and BSR
kernels as the multi-rank chain, without a communicator.  Prints progress per stage (a watchdog
dumps the Python stack after --watchdog seconds).

  python tools/studies/chain_components.py --grid 2 2 1 --Ls 4 --Lt 8 --ncols 12
"""
import argparse
import faulthandler
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import superbblas_amd as sb  # noqa: E402


def log(msg, t0=time.perf_counter()):
    print("chain_components +%.2fs: %s" % (time.perf_counter() - t0, msg), file=sys.stderr,
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, nargs=3, default=[2, 2, 1])
    ap.add_argument("--Ls", type=int, default=4)
    ap.add_argument("--Lt", type=int, default=8)
    ap.add_argument("--ncols", type=int, default=12)
    ap.add_argument("--watchdog", type=float, default=60)
    ap.add_argument("--sync", action="store_true", help="synchronise after every call")
    args = ap.parse_args()
    faulthandler.dump_traceback_later(args.watchdog, exit=True)
    dev = torch.device("cuda", 0)
    grid, Ls, Lt, ncols = args.grid, args.Ls, args.Lt, args.ncols
    nc = grid[0] * grid[1] * grid[2]
    s_, c_ = 4, 3
    b = s_ * c_
    cf = torch.complex64
    G = [Ls * grid[0], Ls * grid[1], Ls * grid[2], Lt]
    dim = G + [s_, c_]
    dsrc = [Lt, ncols, s_, G[0], G[1], G[2], c_]
    # every rank's range of the multi-rank chain, as the components of one process
    psrc = sb.basic_partitioning("tnsxyzc", dsrc, [nc, 1, 1, 1, 1, 1, 1], "t", nc, 1)
    dx = [1] + G + [s_, c_, ncols]
    px = sb.basic_partitioning("pxyztscn", dx, [1] + grid + [1, 1, 1, 1], "xyz", nc, 1)
    src = []
    for f, s in psrc:
        t = torch.empty(bench.vol(s), dtype=cf, device=dev)
        bench.global_fill(t, dsrc, f, s, bench.SEED_SRC)
        src.append(t)
    x = [torch.empty(bench.vol(s), dtype=cf, device=dev) for _, s in px]
    y = [torch.empty_like(t) for t in x]
    pi = sb.basic_partitioning("xyztsc", dim, grid + [1, 1, 1], "xyz", nc, 1)
    pd = []
    for f, sz in pi:
        f, sz = list(f), list(sz)
        for d in range(3):
            if sz[d] + 2 <= dim[d]:
                sz[d] += 2
                f[d] = (f[d] - 1) % dim[d]
            else:
                sz[d], f[d] = dim[d], 0
        pd.append((f, sz))
    iis, jjs, vals = [], [], []
    for c in range(nc):
        f0, s0 = pi[c]
        V = bench.vol(s0[:4])
        sites = np.array(np.unravel_index(np.arange(V), s0[:4])).T + np.array(f0[:4])
        jj = bench.lattice_jj(sites, np.array(G), np.array(pd[c][0][:4]))
        v = torch.empty(V * 9 * b * b, dtype=cf, device=dev)
        bench.global_fill(v, G + [9, b * b], list(f0[:4]) + [0, 0], list(s0[:4]) + [9, b * b],
                          bench.SEED_VALS)
        iis.append(torch.full((V,), 9, dtype=torch.int32, device=dev))
        jjs.append(torch.from_numpy(jj.reshape(-1)).to(dev))
        vals.append(v)
    blk = [1, 1, 1, 1, s_, c_]
    log("create_bsr (%d components, G=%s)" % (nc, G))
    op = sb.create_bsr(pi, dim, pd, dim, blk, blk, False, iis, jjs, vals)

    def sync(what):
        if args.sync:
            torch.cuda.synchronize()
        log(what + " done")

    z7, z8 = [0] * 7, [0] * 8
    log("redistribute")
    sb.copy(1.0, psrc, "tnsxyzc", z7, dsrc, dsrc, src, px, "pxyztscn", z8, dx, x)
    sync("redistribute")
    log("bsr_krylov")
    sb.bsr_krylov(1.0, op, "XYZTSC", "xyztsc", px, "pxyztscn", z8, dx, dx, x, 0.0, px,
                  "pXYZTSCn", z8, dx, dx, "p", y)
    sync("bsr_krylov")
    dr = [Lt, s_, ncols, s_, ncols]
    pr = [([0] * 5, dr)] + [([0] * 5, [0] * 5)] * (nc - 1)
    vr = [torch.empty(bench.vol(dr), dtype=cf, device=dev)] + \
         [torch.empty(1, dtype=cf, device=dev) for _ in range(nc - 1)]
    log("contraction")
    sb.contraction(1.0, px, z8, dx, dx, "pXYZTSCn", True, y, px, z8, dx, dx, "pXYZTsCN", False,
                   y, 0.0, pr, [0] * 5, dr, dr, "TSnsN", vr)
    sync("contraction")
    torch.cuda.synchronize()
    ref = bench.chain_global(sb, dev, G, Lt, ncols)
    err = bench.rel_err(vr[0], ref)
    op.destroy()
    faulthandler.cancel_dump_traceback_later()
    print('{"grid": %s, "G": %s, "rel_err_vs_whole": %.3g}' % (grid, G, err))
    assert err < 1e-5, err


if __name__ == "__main__":
    main()
