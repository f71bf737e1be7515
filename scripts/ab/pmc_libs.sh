#!/bin/bash
# SQ counter passes (one rocprofv3 run per pass) of the cfg2 step kernel for
# each library in LIBS; prints per-wave-step counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmclibs; mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
for L in ${LIBS:-libemcmc}; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/${L}_p$i -o run -- python3 scripts/run_variant.py --lpc ${LPC:-2} --hist full --ll per_obs --steps 200 > $OUT/${L}_p$i.log 2>&1
    rc=$?; echo "$L pass $i rc=$rc"; [ $rc = 0 ] || exit $rc
  done
done
LIBS="${LIBS:-libemcmc}" python3 - <<'PY'
import csv, glob, collections, os
for L in os.environ["LIBS"].split():
    tot = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/pmclibs/{L}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rwm_gsn" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    ws = 2048 * 200 * (2 // int(os.environ.get("LPC", "2")) if False else 1)
    waves = tot.get("SQ_WAVES", 1)
    wsteps = waves * 100  # each wave runs one 100-step launch
    print(L, {k: f"{v / wsteps:.1f}" for k, v in sorted(tot.items()) if k.startswith("SQ_") and k != "SQ_WAVES"}, "waves", waves)
PY
