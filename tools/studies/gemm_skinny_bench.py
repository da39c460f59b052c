#!/usr/bin/env python3
"""tests/dist.cpp's xgemm_batch_strided shapes (test_gemm, tests/dist.cpp:160-195) at its default
lattice (local volume 16*16*16*32*... k = 49152 sites x colors, batch 32): inner products
(m = n = s, k = 49152) and updates (m = 49152, n = k = s), complex<double>, with gemm.frag on and
off (and gemm.skinny), timed by the library's kernel timers (GEMM + split-K reduce).  Reports
TFLOP/s (8 real flops per complex MAC) and the HBM rate of the operand and output bytes.  Not
part of the product.  FRAGS=1,0: the gemm.frag values; SIZES=1,2,4,8,12,16,32,64; DTYPE=cdouble or
cfloat; TALLS: gemm.frag_tall values."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superbblas_amd as sb  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    K, batch = 49152, 32
    sizes = [int(v) for v in os.environ.get("SIZES", "1,2,4,8,12,16,32,64").split(",")]
    frags = [int(v) for v in os.environ.get("FRAGS", "1,0").split(",")]
    # DOTS: gemm.dot_wgs values (m, n <= 4); KINDS: inner,update
    dots = [int(v) for v in os.environ.get("DOTS", str(sb.tune_get("gemm.dot_wgs"))).split(",")]
    kinds = os.environ.get("KINDS", "inner,update").split(",")
    dt = {"cdouble": torch.complex128, "cfloat": torch.complex64}[os.environ.get("DTYPE", "cdouble")]
    es = 16 if dt == torch.complex128 else 8
    talls = [int(v) for v in os.environ.get("TALLS", str(sb.tune_get("gemm.frag_tall"))).split(",")]
    # GEMM_PAIR: gemm.frag_pair (16-byte k pairs for 8-byte elements)
    sb.tune_set("gemm.frag_pair", int(os.environ.get("GEMM_PAIR", "1")))
    # NTS: gemm.frag_nt values (16 x 16 tiles per wave along n)
    nts = [int(v) for v in os.environ.get("NTS", str(sb.tune_get("gemm.frag_nt"))).split(",")]
    # SMALL: gemm.frag_small (the small-output limit of the fragment kernel)
    sb.tune_set("gemm.frag_small", int(os.environ.get("SMALL", str(sb.tune_get("gemm.frag_small")))))
    # FRAGCFG: "uk:waves" pairs for gemm_frag_kernel
    cfgs = [tuple(int(u) for u in v.split(":")) for v in os.environ.get(
        "FRAGCFG", "%d:%d" % (sb.tune_get("gemm.frag_uk"), sb.tune_get("gemm.frag_waves"))).split(",")]
    for kind in kinds:
        for s in sizes:
            m, n, k = (s, s, K) if kind == "inner" else (K, s, s)
            # TA_INNER: the inner products' A form (C: k contiguous, the default; N: m contiguous)
            ta, tb = (os.environ.get("TA_INNER", "C"), "N") if kind == "inner" else ("N", "N")
            lda = k if ta != "N" else m
            a = torch.randn(batch * m * k, dtype=dt, device=dev)
            b = torch.randn(batch * k * n, dtype=dt, device=dev)
            c = torch.zeros(batch * m * n, dtype=dt, device=dev)
            for frag, dot, cfg, tall, nt in [(f, d, c, t, u) for f in frags for d in dots
                                             for c in cfgs for t in talls for u in nts]:
                sb.tune_set("gemm.frag_nt", nt)
                sb.tune_set("gemm.frag", frag)
                sb.tune_set("gemm.frag_tall", tall)
                sb.tune_set("gemm.dot_wgs", dot)
                sb.tune_set("gemm.frag_uk", cfg[0])
                sb.tune_set("gemm.frag_waves", cfg[1])

                def f():
                    sb.xgemm_batch_strided(ta, tb, m, n, k, 1.0, a, lda, m * k, b, k, k * n, 0.0,
                                           c, m, m * n, batch)
                for _ in range(5):
                    f()
                torch.cuda.synchronize()
                ts = []
                for _ in range(3):
                    sb.timings_enable(True)
                    sb.timings_reset()
                    for _ in range(10):
                        f()
                    torch.cuda.synchronize()
                    ms, calls = sb.timings_get("gemm_total")
                    sb.timings_enable(False)
                    ts.append(ms / calls / 1e3)
                t = statistics.median(ts)
                flops = 8.0 * m * n * k * batch
                byts = float(es) * batch * (m * k + k * n + m * n)
                print(json.dumps({"kind": kind, "dtype": str(dt), "m": m, "n": n, "k": k,
                                  "batch": batch, "frag": frag, "frag_tall": tall, "frag_nt": nt, "dot_wgs": dot,
                                  "uk_waves": "%d:%d" % cfg,
                                  "us": round(t * 1e6, 1), "TFLOPs": round(flops / t / 1e12, 3),
                                  "TBps": round(byts / t / 1e12, 3)}), flush=True)
            del a, b, c
    sb.tune_set("gemm.frag", 1)
    sb.tune_set("gemm.frag_uk", 0)
    sb.tune_set("gemm.frag_waves", 4096)
    sb.tune_set("gemm.frag_tall", 0)
    sb.tune_set("gemm.frag_pair", 1)
    sb.tune_set("gemm.frag_nt", 0)
    sb.tune_set("gemm.frag_small", 32)


if __name__ == "__main__":
    main()
