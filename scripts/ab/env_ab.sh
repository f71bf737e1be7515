#!/bin/bash
# Interleaved A/B of runtime environment settings on the driver's 20-step command
# (ENVS: space-separated NAME=VALUE sets, "-" = none); each run under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RTAG:-env_ab}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-3}); do
  for E in ${ENVS:-- HIP_FORCE_DEV_KERNARG=1}; do
    tag=$(echo "$E" | tr '=,' '__')
    f=$OUT/${tag}_r$rep
    if [ "$E" = "-" ]; then envs=(); else IFS=',' read -ra envs <<< "$E"; fi
    env "${envs[@]}" timeout -k 10 300 python3 bench.py ${ARGS:---gpus 1 --steps 20 --warmup 5 --no-cpu} > $f.json 2> $f.err
    rc=$?; [ $rc = 0 ] || { echo "$E rep $rep rc=$rc"; tail -3 $f.err; exit $rc; }
    python3 -c "import json; b=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]); print('$E', '%.4g' % b['value'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), [round(t*1e6,1) for t in b['times_s']][:5])"
  done
done
