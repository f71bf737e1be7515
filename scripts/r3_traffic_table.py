#!/usr/bin/env python3
"""Update profiles/pmc_traffic.json from an r3_roofline_summary.py summary whose
profile directory was copied to profiles/NAME: the measured HBM bytes per timed
launch (WRITE_SIZE + 2 × FETCH_SIZE) of the step kernel at the driver's 20-step
command and the 1000-step default, keyed by launch length, which bench.py reports
as roofline.traffic.  Usage: r3_traffic_table.py profiles/NAME"""
import json
import sys
from pathlib import Path

prof = Path(sys.argv[1])
summ = json.loads((prof / "summary.json").read_text())
table_path = Path(__file__).resolve().parents[1] / "profiles" / "pmc_traffic.json"
table = json.loads(table_path.read_text())
for cfg, cmd in (("s20", "bench.py --gpus 1 --steps 20 --warmup 5"), ("s1000", "bench.py --gpus 1")):
    o = summ.get(cfg)
    if not o or "pmc_traffic" not in o:
        continue
    r = o["bench_roofline"]
    spl = str(int(round(o["bench_line"]["steps"] / r["launches"])))
    pm = o["pmc_traffic"]
    ent = table.setdefault(r["kernel"], {}).setdefault("by_steps_per_launch", {})
    ent[spl] = {"chains": int(round(r["algorithmic_bytes_per_launch"] / r["bytes_per_chain_step"] / int(spl))),
                "traffic_per_launch": pm["traffic_per_launch"],
                "fetch_bytes_x2_per_launch": pm["fetch_bytes_x2_per_launch"],
                "write_bytes_per_launch": pm["write_bytes_per_launch"],
                "algorithmic_per_launch": pm["algorithmic_per_launch"],
                "timed_launches": pm["timed_launches"],
                "command": cmd + " (--no-cpu for the PMC passes)",
                "source": f"{prof}/{cfg}/fetch/run_counter_collection.csv, {prof}/{cfg}/write/run_counter_collection.csv "
                          "(FETCH_SIZE x2 per MI355X_MICROARCH.md HBM section; timed launches only: warm-up and "
                          "clock-settle launches excluded)"}
table_path.write_text(json.dumps(table, indent=1) + "\n")
print(json.dumps({k: list(v.get("by_steps_per_launch", {})) for k, v in table.items()}))
