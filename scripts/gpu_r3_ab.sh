#!/bin/bash
# Interleaved A/B of bench.py argument sets on one box (un-profiled, kernel
# time from HIP events in each line).  ARMS is a '|'-separated list of
# "tag:args" arms; each round runs every arm once, REPS rounds.
#   ARMS="xcd:--no-cpu|noxcd:--no-cpu --variant 16" REPS=3 bash scripts/gpu_r3_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${ABTAG:-ab}
mkdir -p $OUT
IFS='|' read -r -a arms <<< "${ARMS}"
for r in $(seq 1 ${REPS:-3}); do
  for arm in "${arms[@]}"; do
    tag=${arm%%:*}; args=${arm#*:}
    timeout -k 10 ${T_STEP:-300} python3 bench.py $args > $OUT/${tag}_$r.json 2>> $OUT/err.log
    rc=$?
    case $rc in 0) ;; *) echo "arm $tag round $r ended with $rc: stopping"; exit $rc;; esac
    python3 -c "import json,sys; b=json.load(open('$OUT/${tag}_$r.json')); r=b['roofline']; print('$tag', $r, '%.4g'%b['value'], 'kernel %.4g'%b['kernel_chain_steps_per_s'], 'us/step %.3f'%(r['avg_launch_ms']*1e3*r['launches']/b['steps']))"
  done
done
