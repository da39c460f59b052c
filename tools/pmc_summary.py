#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE and WRITE_SIZE collected in separate runs (--pmc FETCH_SIZE / --pmc WRITE_SIZE,
--output-format csv).  Both are in KiB per dispatch; on gfx950 FETCH_SIZE reports half the
bytes of 16-B-per-lane streaming reads (global_load and buffer_load...lds), so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.
Usage: pmc_summary.py fetch.csv write.csv > profiles/rNN_pmc.json"""
import collections
import csv
import json
import re
import sys


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        name = name.replace("HIP_vector_type<double, 2u>", "double2")
        if "sbx::" not in name:
            continue
        agg[name.split("(sbx::")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(fetch_csv, write_csv):
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    out = {}
    for k in sorted(set(f) | set(w)):
        rb = 2 * 1024.0 * f.get(k, 0.0)
        wb = 1024.0 * w.get(k, 0.0)
        out[k] = {"read_bytes": rb, "write_bytes": wb, "hbm_bytes": rb + wb}
    json.dump({"method": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes), "
                         "FETCH_SIZE x2 (gfx950 16-B/lane read correction), KiB -> bytes, "
                         "average per dispatch", "kernels": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
