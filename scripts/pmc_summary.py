#!/usr/bin/env python3
"""Summarise a profile_round.sh directory: per-kernel average durations from the
kernel trace and HBM traffic per launch of the step kernel from FETCH_SIZE /
WRITE_SIZE (KiB units; FETCH_SIZE ×2 on gfx950 per MI355X_MICROARCH.md §HBM)."""
import csv
import glob
import json
import re
import sys

# step kernels: fused RWM (rwm_gsn_*) and mix / chain-moments (mix_gsn_kernel)
STEP = re.compile(r"rwm_gsn|mix_gsn_kernel")
from collections import defaultdict

d = sys.argv[1]


def rows(pattern):
    out = []
    for f in glob.glob(f"{d}/{pattern}", recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


stats = {r["Name"]: {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "total_ns": float(r["TotalDurationNs"]),
                     "pct": float(r["Percentage"])} for r in rows("trace/**/*kernel_stats.csv")}
step = [k for k in stats if STEP.search(k)]
res = {"kernel_stats": stats}
pmc = defaultdict(list)
for name in ("FETCH_SIZE", "WRITE_SIZE"):
    sub = "fetch" if name == "FETCH_SIZE" else "write"
    for r in rows(f"{sub}/**/*counter_collection.csv"):
        if STEP.search(r["Kernel_Name"]) and r["Counter_Name"] == name:
            pmc[name].append(float(r["Counter_Value"]))
if pmc:
    f = pmc["FETCH_SIZE"]
    w = pmc["WRITE_SIZE"]
    # the timed launches are the last ones (warmup launch first)
    res["pmc"] = {"fetch_kib_per_launch": f, "write_kib_per_launch": w,
                  "fetch_bytes_corrected_per_launch": [2 * 1024 * x for x in f],
                  "write_bytes_per_launch": [1024 * x for x in w]}
print(json.dumps(res, indent=1))
