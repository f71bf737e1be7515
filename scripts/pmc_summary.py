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
by_kernel = defaultdict(lambda: defaultdict(list))
GROUP = re.compile(r"mix_gsn_kernel|mix_moments_kernel|mix_readjust_kernel")
for name in ("FETCH_SIZE", "WRITE_SIZE"):
    sub = "fetch" if name == "FETCH_SIZE" else "write"
    for r in rows(f"{sub}/**/*counter_collection.csv"):
        if r["Counter_Name"] != name:
            continue
        if STEP.search(r["Kernel_Name"]):
            pmc[name].append(float(r["Counter_Value"]))
        if GROUP.search(r["Kernel_Name"]):
            by_kernel[r["Kernel_Name"]][name].append(float(r["Counter_Value"]))
if pmc:
    f = pmc["FETCH_SIZE"]
    w = pmc["WRITE_SIZE"]
    # the timed launches are the last ones (warmup launch first)
    res["pmc"] = {"fetch_kib_per_launch": f, "write_kib_per_launch": w,
                  "fetch_bytes_corrected_per_launch": [2 * 1024 * x for x in f],
                  "write_bytes_per_launch": [1024 * x for x in w]}
if by_kernel:
    # mix path: HBM bytes of the whole launch group (step + moments + readjust)
    # per step-kernel launch, FETCH_SIZE x2 as above
    nstep = max(len(v["FETCH_SIZE"]) for k, v in by_kernel.items() if "mix_gsn_kernel" in k)
    tot_f = sum(2 * 1024 * sum(v["FETCH_SIZE"]) for v in by_kernel.values())
    tot_w = sum(1024 * sum(v["WRITE_SIZE"]) for v in by_kernel.values())
    res["group"] = {"kernels": {k: {"fetch_bytes_corrected": 2 * 1024 * sum(v["FETCH_SIZE"]),
                                    "write_bytes": 1024 * sum(v["WRITE_SIZE"]), "launches": len(v["FETCH_SIZE"])}
                                for k, v in by_kernel.items()},
                    "step_launches": nstep, "fetch_bytes_corrected_per_group": tot_f / nstep,
                    "write_bytes_per_group": tot_w / nstep}
print(json.dumps(res, indent=1))
