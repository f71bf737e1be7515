#!/usr/bin/env python3
"""Summarise scripts/gpu_r3_roofline.sh: for the driver's 20-step command and the
1000-step default, the step kernel's timed launches from the rocprofv3 kernel
trace, the roofline fraction they give against the bench line's own, the HBM
traffic per timed launch (WRITE_SIZE + 2 × FETCH_SIZE, KiB units;
MI355X_MICROARCH.md HBM section) and the effective clock (GRBM_GUI_ACTIVE / 8 /
duration, its "DVFS give-back" note); then the gap experiments' lines.
Usage: r3_roofline_summary.py DIR"""
import csv
import glob
import json
import math
import re
import sys

STEP = re.compile(r"rwm_gsn|mix_res_kernel|mix_gsn_kernel|mala_logistic_kernel")
d = sys.argv[1]


def line(path):
    try:
        for ln in reversed(open(path).read().strip().split("\n")):
            if ln.startswith("{"):
                return json.loads(ln)
    except OSError:
        pass
    return None


def rows(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        out += list(csv.DictReader(open(f)))
    return out


def timed_slice(b, n_dispatch):
    """Indices of the timed launches: warm-up launches first, then the clock-settle
    launches of the throwaway handle (bench.py settle_clock), then reps × launches per rep."""
    spl = b["config"]["steps_per_launch"]
    nw = math.ceil(b["warmup"] / spl) if b["warmup"] else 0
    nw += (b["config"].get("clock_settle") or {}).get("launches", 0)
    per = b["roofline"]["launches"]
    # round 4: each value rep is followed by a kernel-timing rep (bench.py kernel_timing_reps)
    reps = b["reps"] + ((b.get("kernel_timing_reps") or {}).get("n") or 0)
    return nw, min(n_dispatch, nw + reps * per)


res = {}
for cfg in ("s20", "s1000"):
    b = line(f"{d}/{cfg}/trace.json")
    if b is None:
        continue
    out = {"bench_line": {k: b[k] for k in ("value", "steps", "warmup", "reps", "kernel_chain_steps_per_s")},
           "bench_roofline": b["roofline"]}
    tr = [r for r in rows(f"{d}/{cfg}/trace/**/*kernel_trace.csv") if STEP.search(r["Kernel_Name"])]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr]
    a, z = timed_slice(b, len(dur))
    timed = dur[a:z]
    bytes_per_launch = b["roofline"]["algorithmic_bytes_per_launch"]
    if timed:
        avg = sum(timed) / len(timed)
        out["rocprof_trace"] = {"kernel": tr[0]["Kernel_Name"], "dispatches": len(dur), "timed_dispatches": [a, z],
                                "timed_avg_ns": avg, "timed_ns": timed, "all_ns": dur,
                                "achieved_GBs": bytes_per_launch / avg, "frac": bytes_per_launch / avg / 8000.0,
                                "frac_vs_bench_line": (bytes_per_launch / avg / 8000.0) / b["roofline"]["frac"]}
    pm = {}
    for sub, name in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        rr = [r for r in rows(f"{d}/{cfg}/{sub}/**/*counter_collection.csv")
              if r["Counter_Name"] == name and STEP.search(r["Kernel_Name"])]
        rr.sort(key=lambda r: int(r["Dispatch_Id"]))
        a2, z2 = timed_slice(line(f"{d}/{cfg}/{sub}.json") or b, len(rr))  # that pass's own settle launches
        pm[name] = [float(r["Counter_Value"]) for r in rr[a2:z2]]
    if pm.get("FETCH_SIZE") and pm.get("WRITE_SIZE"):
        f = sum(pm["FETCH_SIZE"]) / len(pm["FETCH_SIZE"]) * 1024 * 2
        w = sum(pm["WRITE_SIZE"]) / len(pm["WRITE_SIZE"]) * 1024
        out["pmc_traffic"] = {"fetch_bytes_x2_per_launch": f, "write_bytes_per_launch": w,
                              "traffic_per_launch": f + w, "algorithmic_per_launch": bytes_per_launch,
                              "traffic_over_algorithmic": (f + w) / bytes_per_launch,
                              "timed_launches": len(pm["WRITE_SIZE"])}
    ck = rows(f"{d}/{cfg}/clock/**/*counter_collection.csv")
    if ck:
        by = {}
        for r in ck:
            if not STEP.search(r["Kernel_Name"]):
                continue
            e = by.setdefault(int(r["Dispatch_Id"]), {"ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        ds = [by[k] for k in sorted(by)]
        a3, z3 = timed_slice(line(f"{d}/{cfg}/clock.json") or b, len(ds))
        ds = ds[a3:z3]
        if ds:
            clk = [e["GRBM_GUI_ACTIVE"] / 8 / e["ns"] for e in ds if "GRBM_GUI_ACTIVE" in e]
            out["clock"] = {"effective_ghz_per_timed_launch": clk, "mean_ghz": sum(clk) / len(clk),
                            "timed_launch_ns": [e["ns"] for e in ds],
                            "sq_wave_cycles_per_wave": [e.get("SQ_WAVE_CYCLES", 0) / max(1, e.get("SQ_WAVES", 1))
                                                        for e in ds],
                            "note": "GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time; reads high below ~0.3 ms"}
    res[cfg] = out
gap = {}
for f in sorted(glob.glob(f"{d}/gap_*.json")):
    b = line(f)
    if b is None:
        continue
    r = b["roofline"]
    spl_eff = b["steps"] / r["launches"]
    gap[f.split("/")[-1][:-5]] = {"value": b["value"], "kernel_chain_steps_per_s": b["kernel_chain_steps_per_s"],
                                  "avg_launch_ms": r["avg_launch_ms"], "steps_per_launch": spl_eff,
                                  "us_per_step_in_kernel": r["avg_launch_ms"] * 1e3 / spl_eff, "frac": r["frac"],
                                  "steps": b["steps"], "warmup": b["warmup"], "reps": b["reps"]}
res["gap_experiments"] = gap
print(json.dumps(res, indent=1))
