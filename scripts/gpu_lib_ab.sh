#!/bin/bash
# Interleaved A/B of libemcmc builds on one box: LIBS="tag:path|tag:path"
# (path empty = the in-tree default), the same bench.py ARGS for every arm.
#   LIBS="base:|w16:extensiblemcmc.jl_amd/lib/ab/libemcmc_w16.so" ARGS="--workload cfg4 --no-cpu" bash scripts/gpu_lib_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${ABTAG:-libab}
mkdir -p $OUT
IFS='|' read -r -a libs <<< "${LIBS}"
for r in $(seq 1 ${REPS:-3}); do
  for arm in "${libs[@]}"; do
    tag=${arm%%:*}; lib=${arm#*:}
    if [ -n "$lib" ]; then export EMCMC_LIB=$PWD/$lib; else unset EMCMC_LIB; fi
    timeout -k 10 ${T_STEP:-300} python3 bench.py $ARGS > $OUT/${tag}_$r.json 2>> $OUT/err.log
    rc=$?
    case $rc in 0) ;; *) echo "arm $tag round $r ended with $rc: stopping"; exit $rc;; esac
    python3 -c "import json; b=json.load(open('$OUT/${tag}_$r.json')); r=b['roofline']; print('$tag', $r, '%.4g'%b['value'], 'kernel %.4g'%b['kernel_chain_steps_per_s'], 'ms/launch %.3f'%r['avg_launch_ms'])"
  done
done
