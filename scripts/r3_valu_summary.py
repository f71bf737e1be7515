#!/usr/bin/env python3
"""Compute roofline of the cfg 4 launch group from a rocprofv3 --pmc pass of
SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64, SQ_ACTIVE_INST_VALU, SQ_INSTS_VALU,
SQ_WAVES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE (scripts/gpu_r3_cfgs.sh): per kernel,
averaged over its dispatches, the fp64 VALU rate (64 lanes × (2·FMA + MUL + ADD)
per wave-instruction; full EXEC assumed), the VALU-issue fraction
(SQ_ACTIVE_INST_VALU quad-cycles × 4 / 1,024 SIMDs / (GRBM_GUI_ACTIVE / 8)), the
effective clock and the fp64 rate against the VALU peak at that clock and at
2.4 GHz (78.6 TFLOP/s).  Usage: r3_valu_summary.py COUNTER_CSV"""
import csv
import json
import re
import sys
from collections import defaultdict

PEAK = 78.6  # TFLOP/s fp64 vector, 256 CUs × 4 SIMDs × 16 fma lanes × 2 × 2.4 GHz
KERN = re.compile(r"mix_res_kernel|mix_moments_kernel|mix_readjust_kernel|mix_gsn_kernel|rwm_gsn|mala_logistic")
agg = defaultdict(lambda: defaultdict(float))
dur = {}
for r in csv.DictReader(open(sys.argv[1])):
    if not KERN.search(r["Kernel_Name"]):
        continue
    k = (re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void emcmc::", ""), int(r["Dispatch_Id"]))
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    dur[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
per = defaultdict(list)
for k, c in agg.items():
    per[k[0]].append((dur[k], c))
out = {}
for name, ds in per.items():
    ns = sum(d for d, _ in ds) / len(ds)
    tot = defaultdict(float)
    for _, c in ds:
        for n, v in c.items():
            tot[n] += v / len(ds)
    flop = 64 * (2 * tot["SQ_INSTS_VALU_FMA_F64"] + tot["SQ_INSTS_VALU_MUL_F64"] + tot["SQ_INSTS_VALU_ADD_F64"])
    ghz = tot["GRBM_GUI_ACTIVE"] / 8 / ns
    tfs = flop / ns / 1e3
    out[name] = {"dispatches": len(ds), "avg_ns": ns, "fp64_flop_per_dispatch": flop, "fp64_tflops": tfs,
                 "fp64_frac_of_peak": tfs / PEAK, "fp64_frac_of_peak_at_clock": tfs / (PEAK * ghz / 2.4),
                 "effective_ghz": ghz,
                 "valu_busy": tot["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (tot["GRBM_GUI_ACTIVE"] / 8),
                 "valu_insts_per_wave": tot["SQ_INSTS_VALU"] / max(1.0, tot["SQ_WAVES"]),
                 "f64_share_of_valu": (tot["SQ_INSTS_VALU_FMA_F64"] + tot["SQ_INSTS_VALU_MUL_F64"] +
                                       tot["SQ_INSTS_VALU_ADD_F64"] + tot["SQ_INSTS_VALU_TRANS_F64"]) /
                                      max(1.0, tot["SQ_INSTS_VALU"]),
                 "counters_avg": dict(tot)}
print(json.dumps(out, indent=1))
