#!/usr/bin/env python3
"""Per-dispatch PMC counter table for the kernels whose name contains a substring, from a
rocprofv3 --pmc csv (tools only).  Usage: pmc_kernels.py run_counter_collection.csv substr"""
import collections
import csv
import sys


def main(path, sub):
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if sub not in r["Kernel_Name"]:
            continue
        key = (int(r["Dispatch_Id"]), r["Counter_Name"])
        agg[key] = agg.get(key, 0) + float(r["Counter_Value"])
    for d in sorted(set(k[0] for k in agg)):
        names = sorted(n for (dd, n) in agg if dd == d)
        print(d, {n: round(agg[(d, n)]) for n in names})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
