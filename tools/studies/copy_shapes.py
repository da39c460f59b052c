#!/usr/bin/env python3
"""Time the box-copy kernel on named permutations (not part of the product):
  slice  xyztsc -> tnsxyzc[n]        (config 2p, one slice, complex<double>)
  big    xyztnsc -> tnsxyzc          (whole tensor, complex<double>)
  chain  pXYZTSCn -> TSnpXYZC        (the chain's contraction operand reorder, complex<float>)
kernel time from the library timers; SBX_COPY_DEBUG=1 prints the tiling."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def vol(d):
    n = 1
    for x in d:
        n *= x
    return n


def case(name, o0, d0, o1, d1, from1, dtype, reps=10):
    dev = torch.device("cuda:0")
    dtype, dtype_out = dtype if isinstance(dtype, tuple) else (dtype, dtype)
    a = torch.randn(vol(d0), dtype=dtype, device=dev)
    b = torch.zeros(vol(d1), dtype=dtype_out, device=dev)
    p0, p1 = [([0] * len(d0), d0)], [([0] * len(d1), d1)]

    def f():
        sb.copy(1.0, p0, o0, [0] * len(d0), d0, d0, [a], p1, o1, from1, d1, [b])
    f()
    torch.cuda.synchronize()
    sb.timings_enable(True)
    sb.timings_reset()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    ms, calls = sb.timings_get("copy")
    sb.timings_enable(False)
    t = ms / calls / 1e3
    es = torch.empty(0, dtype=dtype).element_size()
    ok = bool(torch.equal(b.view(-1), ref_copy(a.to(dtype_out), o0, d0, o1, d1, from1).view(-1)))
    eo = torch.empty(0, dtype=dtype_out).element_size()
    print(json.dumps({"case": name, "us": round(t * 1e6, 1),
                      "GBps": round((es + eo) * vol(d0) / t / 1e9, 1), "exact": ok,
                      "kind": sb.tune_get("copy.last_pair")}))


def ref_copy(a, o0, d0, o1, d1, from1):
    """torch permute of the whole source into the destination box (full-size check)"""
    src = a.view(*d0)
    perm = [o0.index(c) for c in o1 if c in o0]
    out = torch.zeros(d1, dtype=a.dtype, device=a.device)
    sl = tuple(slice(f, f + (d0[o0.index(c)] if c in o0 else 1)) for c, f in zip(o1, from1))
    view = src.permute(*perm)
    out[sl] = view.reshape(out[sl].shape)
    return out


def sweep(spec):
    """COPY_SWEEP="budget:run,...": tile budget / source-run target on the chain-sized cases"""
    for item in spec.split(","):
        budget, run = (int(v) for v in item.split(":"))
        sb.tune_set("copy.budget", budget)
        sb.tune_set("copy.run", run)
        print(json.dumps({"copy.budget": budget, "copy.run": run}))
        L, n = 16, 64
        case("redist", "tnsxyzc", [64, 12, 4, 16, 16, 16, 3], "pxyztscn",
             [1, 16, 16, 16, 64, 4, 3, 12], [0] * 8, torch.complex64)
        case("chain", "pXYZTSCn", [1, 16, 16, 16, 64, 4, 3, 12], "TSnpXYZC",
             [64, 4, 12, 1, 16, 16, 16, 3], [0] * 8, torch.complex64)
        case("big", "xyztnsc", [L, L, L, L, n, 4, 3], "tnsxyzc", [L, n, 4, L, L, L, 3], [0] * 7,
             torch.complex128)
    sb.tune_set("copy.budget", 0)
    sb.tune_set("copy.run", 0)


def kinds():
    """COPY_KINDS=1: the transpose kernels on / off on every case (copy.trans, copy.btrans)"""
    for trans, btrans in ((0, 0), (0, -1), (-1, -1)):
        sb.tune_set("copy.trans", trans)
        sb.tune_set("copy.btrans", btrans)
        print(json.dumps({"copy.trans": trans, "copy.btrans": btrans}))
        shapes()
    sb.tune_set("copy.trans", 0)
    sb.tune_set("copy.btrans", 0)


def main():
    if os.environ.get("COPY_SWEEP"):
        return sweep(os.environ["COPY_SWEEP"])
    if os.environ.get("COPY_KINDS"):
        return kinds()
    if os.environ.get("COPY_MID"):
        return mid()
    combos = ((0, 0, 0), (0, 0, -1), (0, 0, -2), (0, -1, 0))
    if os.environ.get("COPY_QUICK"):
        combos = combos[:3]
    for kern, nt, pair in combos:
        sb.tune_set("copy.nt", nt)
        sb.tune_set("copy.pair", 0 if pair == -2 else pair)
        sb.tune_set("copy.order", -1 if pair == -2 else 0)  # -2: pairs, destination chain first
        print(json.dumps({"copy.nt": nt, "copy.pair": pair}))
        shapes()
    sb.tune_set("copy.nt", 0)
    sb.tune_set("copy.pair", 0)
    sb.tune_set("copy.order", 0)


def mid():
    """COPY_MID=1: 4-8 MB outputs (under the 8 MB streaming-store threshold of the block and tile
    kernels) with streaming stores off / on, twice"""
    for nt in (0, 1, 0, 1):
        sb.tune_set("copy.nt", nt if nt else 0)
        print(json.dumps({"copy.nt": nt}))
        case("redist_mid", "tnsxyzc", [4, 12, 4, 8, 8, 16, 3], "pxyztscn",
             [1, 8, 8, 16, 4, 4, 3, 12], [0] * 8, torch.complex64, reps=50)
        case("chain_mid", "pXYZTSCn", [1, 8, 8, 16, 4, 4, 3, 12], "TSnpXYZC",
             [4, 4, 12, 1, 8, 8, 16, 3], [0] * 8, torch.complex64, reps=50)
        case("big_mid", "xyztnsc", [8, 8, 8, 8, 16, 4, 3], "tnsxyzc", [8, 16, 4, 8, 8, 8, 3],
             [0] * 7, torch.complex64, reps=50)
    sb.tune_set("copy.nt", 0)


def shapes():
    L, n = 16, 64
    case("slice", "xyztsc", [L, L, L, L, 4, 3], "tnsxyzc", [L, n, 4, L, L, L, 3],
         [0, 5, 0, 0, 0, 0, 0], torch.complex128)
    case("big", "xyztnsc", [L, L, L, L, n, 4, 3], "tnsxyzc", [L, n, 4, L, L, L, 3], [0] * 7,
         torch.complex128)
    case("redist", "tnsxyzc", [64, 12, 4, 16, 16, 16, 3], "pxyztscn",
         [1, 16, 16, 16, 64, 4, 3, 12], [0] * 8, torch.complex64)
    case("chain", "pXYZTSCn", [1, 16, 16, 16, 64, 4, 3, 12], "TSnpXYZC",
         [64, 4, 12, 1, 16, 16, 16, 3], [0] * 8, torch.complex64)
    case("slice_cf", "xyztsc", [L, L, L, L, 4, 3], "tnsxyzc", [L, n, 4, L, L, L, 3],
         [0, 5, 0, 0, 0, 0, 0], torch.complex64)
    case("big_cf", "xyztnsc", [L, L, L, L, n, 4, 3], "tnsxyzc", [L, n, 4, L, L, L, 3], [0] * 7,
         torch.complex64)
    case("slice_cf2cd", "xyztsc", [L, L, L, L, 4, 3], "tnsxyzc", [L, n, 4, L, L, L, 3],
         [0, 5, 0, 0, 0, 0, 0], (torch.complex64, torch.complex128))
    case("big_f64", "xyztnsc", [L, L, L, L, n, 4, 3], "tnsxyzc", [L, n, 4, L, L, L, 3], [0] * 7,
         torch.float64)


if __name__ == "__main__":
    main()
