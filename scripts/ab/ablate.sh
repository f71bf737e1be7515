#!/bin/bash
# Timing-only ablation sweep of the cfg2 step kernel (FULL, PER_OBS, LPC=2):
# base vs cheap-hash RNG (ABL=1), no rare paths (ABL=2), both (ABL=3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ablate; mkdir -p $OUT
for A in 0 ${ABLS:-1 2 3}; do
  LIBF=extensiblemcmc.jl_amd/lib/libemcmc.so; [ $A = 0 ] || LIBF=extensiblemcmc.jl_amd/lib/libemcmc_ablate$A.so
  EMCMC_LIB=$PWD/$LIBF timeout -k 10 300 python scripts/kbench.py --grid 2:0 --hist full --ll ${LL:-per_obs} --rounds 3 --steps 300 > $OUT/abl$A.json 2> $OUT/abl$A.err
  rc=$?; echo "ABL=$A rc=$rc $(cat $OUT/abl$A.json)"; case $rc in 0) ;; *) exit $rc;; esac
done
