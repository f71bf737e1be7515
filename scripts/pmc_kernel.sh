#!/bin/bash
# PMC passes (one rocprofv3 run per pass) of CMD, summed per kernel whose
# name matches KRE; prints per-launch counter values.
#   KRE=mix_moments CMD="python3 bench.py --workload cfg4 --no-cpu --steps 200 --warmup 0" bash scripts/pmc_kernel.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmck_${TAG:-x}; mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
P5="TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc = 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
KRE="$KRE" OUT="$OUT" python3 - <<'PY'
import csv, glob, collections, os, re
kre = re.compile(os.environ["KRE"]); out = os.environ["OUT"]
tot = collections.defaultdict(lambda: collections.defaultdict(float)); calls = collections.defaultdict(set)
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kre.search(r["Kernel_Name"]):
            k = r["Kernel_Name"][:60]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add((f.split('/p')[1][:1], r.get("Dispatch_Id", r.get("Correlation_Id", ""))))
for k, d in tot.items():
    n = max(1, len([c for c in calls[k] if c[0] == '1']))
    print(k, "launches", n, {c: f"{v / n:.4g}" for c, v in sorted(d.items())})
PY
