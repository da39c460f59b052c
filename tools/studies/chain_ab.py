#!/usr/bin/env python3
"""A/B of library tune settings on the bench's configs[4] chain (bench.chain_bench: redistribute
-> 12x12 BSR -> contraction, 16^3 x 64 sites, complex<float>), the settings interleaved in one
process so box-to-box and clock drift cancel.  Not part of the product.

  AB='bsr.nt=11;bsr.nt=10' ROUNDS=4 python tools/studies/chain_ab.py
(each setting a comma-separated list of key=value; every key is restored after its run)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import superbblas_amd as sb  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    settings = [[kv.split("=") for kv in s.split(",") if kv]
                for s in os.environ.get("AB", "bsr.nt=11;bsr.nt=10").split(";")]
    rounds = int(os.environ.get("ROUNDS", "4"))
    for r in range(rounds):
        for st in settings:
            old = [(k, sb.tune_get(k)) for k, _ in st]
            for k, v in st:
                sb.tune_set(k, int(v))
            try:
                res = bench.chain_bench(sb, dev)
            finally:
                for k, v in old:
                    sb.tune_set(k, v)
            print(json.dumps({"round": r, "setting": ",".join("%s=%s" % (k, v) for k, v in st),
                              **{k: res[k] for k in ("chain_ms", "chain_redistribute_ms",
                                                     "chain_bsr_ms", "chain_contraction_ms")}}),
                  flush=True)


if __name__ == "__main__":
    main()
