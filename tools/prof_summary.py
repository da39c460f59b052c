#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats database (rocpd sqlite) into a text table:
per kernel the number of calls, total/average/median/min/max duration (us) and share of GPU time.
The median is the figure to quote: a single dispatch stalled by the tracer (a 14-18 ms outlier
seen under rocprofv3 only) moves the average of a short kernel, not its median.
Usage: prof_summary.py run_results.db [> profiles/<name>.txt]"""
import re
import sqlite3
import statistics
import sys


def short(name, width=110):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = name.replace("HIP_vector_type<double, 2u>", "double2")
    name = name.replace("HIP_vector_type<float, 2u>", "float2")
    if name.startswith("void at::native"):
        name = name.split("<")[0] + "<...>"
    return name if len(name) <= width else name[:width - 3] + "..."


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(end - start), avg(end - start), min(end - start), "
        "max(end - start) from kernels group by name order by sum(end - start) desc").fetchall()
    durs = {}
    for name, d in c.execute("select name, end - start from kernels"):
        durs.setdefault(name, []).append(d)
    tot = sum(r[2] for r in rows) or 1
    print("%-110s %6s %12s %10s %10s %10s %10s %6s" % ("kernel", "calls", "total_us", "avg_us",
                                                       "median_us", "min_us", "max_us", "pct"))
    for name, n, s, a, mi, ma in rows:
        med = statistics.median(durs[name])
        print("%-110s %6d %12.1f %10.2f %10.2f %10.2f %10.2f %6.2f" % (
            short(name), n, s / 1e3, a / 1e3, med / 1e3, mi / 1e3, ma / 1e3, 100.0 * s / tot))


if __name__ == "__main__":
    main(sys.argv[1])
