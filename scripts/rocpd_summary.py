#!/usr/bin/env python3
"""Summaries of rocprofv3 output for profiles/: a kernel-trace database (run_results.db,
rocprofv3 7.2's default format) → per-kernel calls / total / average ns plus the dispatch
resources (VGPRs, AGPRs, scratch bytes per lane, LDS); a --pmc counter_collection.csv →
per-kernel counter sums per dispatch.

  python3 scripts/rocpd_summary.py trace gpurun_out/x/kt/run_results.db > profiles/y/kernel_stats.csv
  python3 scripts/rocpd_summary.py pmc gpurun_out/x/pmc/run_counter_collection.csv > profiles/y/pmc.csv
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def trace(db):
    con = sqlite3.connect(db)
    rows = con.execute(
        "select name, count(*), sum(duration), avg(duration), max(vgpr_count), max(accum_vgpr_count), "
        "max(scratch_size), max(lds_size), max(sgpr_count) from kernels group by name order by sum(duration) desc"
    ).fetchall()
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "total_ns", "avg_ns", "vgprs", "agprs", "scratch_bytes_per_lane", "lds_bytes",
                "sgprs"])
    for r in rows:
        w.writerow([r[0], r[1], f"{r[2]:.0f}", f"{r[3]:.1f}", *r[4:]])


def pmc(path):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row.get("Kernel_Name") or row.get("Kernel-Name") or row.get("kernel_name")
            c = row.get("Counter_Name") or row.get("Counter-Name")
            v = float(row.get("Counter_Value") or row.get("Counter-Value") or 0)
            d = row.get("Dispatch_Id") or row.get("Dispatch-Id") or row.get("Correlation_Id")
            acc[k][c] += v
            disp[k].add(d)
    names = sorted({c for k in acc for c in acc[k]})
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "dispatches"] + [f"{c}_per_dispatch" for c in names])
    for k in sorted(acc, key=lambda k: -sum(acc[k].values())):
        n = max(1, len(disp[k]))
        w.writerow([k, n] + [f"{acc[k].get(c, 0.0) / n:.6g}" for c in names])


if __name__ == "__main__":
    {"trace": trace, "pmc": pmc}[sys.argv[1]](sys.argv[2])
