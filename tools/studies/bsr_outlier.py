#!/usr/bin/env python3
"""Per-launch durations of the config-3 n = 64 BSR product (bsr_ell9_kernel) without a profiler
attached (not part of the product): the bench's warm-up loop shape (launch, synchronise) repeated
N times, each launch bracketed by its own HIP event pair on the launch stream.  Prints the
median, the maximum and every launch above 5x the median, to tell whether the 14 ms dispatch seen
twice under rocprofv3 --kernel-trace also happens in a plain run."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import superbblas_amd as sb  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    ncols = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    dev = torch.device("cuda:0")
    L = 16
    op, x, y, run = bench.bsr_setup(sb, dev, L, ncols)
    stream = torch.cuda.current_stream()
    for _ in range(20):
        run()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(n)]
    for s, e in evs:
        s.record(stream)
        run()
        e.record(stream)
        torch.cuda.synchronize()
    d = [s.elapsed_time(e) * 1e3 for s, e in evs]
    med = statistics.median(d)
    out = [(i, round(v, 1)) for i, v in enumerate(d) if v > 5 * med]
    print(json.dumps({"ncols": ncols, "launches": n, "median_us": round(med, 1),
                      "max_us": round(max(d), 1), "outliers_over_5x_median": out}), flush=True)
    op.destroy()


if __name__ == "__main__":
    main()
