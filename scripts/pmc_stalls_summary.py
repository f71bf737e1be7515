#!/usr/bin/env python3
"""Per-kernel wave-time split from one rocprofv3 --pmc pass (scripts/gpu_r6_stalls.sh):
SQ_WAIT_ANY (parked on s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stall) and
SQ_ACTIVE_INST_ANY (issuing) as fractions of SQ_WAVE_CYCLES (MI355X_MICROARCH.md: disjoint, all in
quad-cycles), VALU / scalar issue shares, instructions per wave.
  python3 scripts/pmc_stalls_summary.py <run_counter_collection.csv> [...]"""
import csv
import json
import sys
from collections import defaultdict


def summarize(path):
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    waves = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if k.startswith("__amd"):
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
        waves[k] = int(r["Grid_Size"]) // 64
    out = {}
    for k, c in acc.items():
        d = len(n[k])
        wc = c["SQ_WAVE_CYCLES"] or 1.0
        out[k[:110]] = {
            "dispatches": d,
            "wait_any": round(c["SQ_WAIT_ANY"] / wc, 3),
            "wait_inst_any": round(c["SQ_WAIT_INST_ANY"] / wc, 3),
            "active_inst_any": round(c["SQ_ACTIVE_INST_ANY"] / wc, 3),
            "active_valu": round(c["SQ_ACTIVE_INST_VALU"] / wc, 3),
            "active_scalar": round(c["SQ_ACTIVE_INST_SCA"] / wc, 3),
            "valu_insts_per_wave_dispatch": round(c["SQ_INSTS_VALU"] / d / waves[k], 1),
            "smem_insts_per_wave_dispatch": round(c["SQ_INSTS_SMEM"] / d / waves[k], 1),
        }
    return out


if __name__ == "__main__":
    res = {}
    for p in sys.argv[1:]:
        res.update(summarize(p))
    print(json.dumps(res, indent=1))
