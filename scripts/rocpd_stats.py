#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 rocpd database (the default output format): one CSV row per
kernel name with calls, total / average / min / max duration (ns), share of the total, and the
dispatch records' VGPR, AGPR, SGPR counts and scratch bytes per lane.
  python3 scripts/rocpd_stats.py <results.db> > kernel_stats.csv"""
import csv
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(scratch_size) from kernels "
        "group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage", "VGPR", "AGPR",
                "SGPR", "ScratchPerLane"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5], round(100.0 * r[2] / total, 3)] + list(r[6:]))


if __name__ == "__main__":
    main(sys.argv[1])
