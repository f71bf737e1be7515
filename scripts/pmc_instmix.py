#!/usr/bin/env python3
"""Per-kernel instruction mix per dispatch from one rocprofv3 --pmc directory:
  python scripts/pmc_instmix.py DIR OUT.csv
(counter_collection.csv rows summed per dispatch, averaged over the dispatches of
each kernel).  SQ_INSTS_FLAT counts the scratch (private-segment) accesses of a
kernel whose arrays spill or are dynamically indexed."""
import collections
import csv
import glob
import sys

d, out = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
names = sorted({c for v in acc.values() for c in v})
with open(out, "w", newline="") as fo:
    w = csv.writer(fo)
    w.writerow(["kernel", "dispatches"] + [f"{c}_per_dispatch" for c in names])
    for k, v in sorted(acc.items()):
        n = max(1, len(disp[k]))
        w.writerow([k, n] + [f"{v[c] / n:.6g}" for c in names])
print(open(out).read())
