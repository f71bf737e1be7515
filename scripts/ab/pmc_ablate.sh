#!/bin/bash
# SQ counter passes (one rocprofv3 run per pass) of the cfg2 step kernel for
# the base build and the no-rare-path timing build (ABL=2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcab; mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
P3="SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_BUSY_CYCLES"
for A in ${ABLS:-0 2}; do
  LIBF=extensiblemcmc.jl_amd/lib/libemcmc.so; [ $A = 0 ] || LIBF=extensiblemcmc.jl_amd/lib/libemcmc_ablate$A.so
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    EMCMC_LIB=$PWD/$LIBF timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/a${A}p$i -o run -- python3 scripts/run_variant.py --lpc 2 --hist full --ll per_obs --steps 200 > $OUT/a${A}p$i.log 2>&1
    rc=$?; echo "A=$A pass $i rc=$rc"; [ $rc = 0 ] || exit $rc
  done
done
python3 - <<'PY'
import csv, glob, collections
for A in (0, 2):
    tot = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/pmcab/a{A}p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rwm_gsn" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print("ABL", A, {k: f"{v:.4g}" for k, v in sorted(tot.items())})
PY
