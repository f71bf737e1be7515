#!/bin/bash
# Interleaved A/B of library builds (LIBS, in extensiblemcmc.jl_amd/lib/) on bench.py
# command lines (ARGSETS, ';'-separated); REPS rounds; each run under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RTAG:-lib_ab}
mkdir -p $OUT
IFS=';' read -ra SETS <<< "${ARGSETS:---gpus 1 --steps 20 --warmup 5 --no-cpu}"
for rep in $(seq 1 ${REPS:-3}); do
  for si in "${!SETS[@]}"; do
    for L in ${LIBS:-libemcmc_base libemcmc}; do
      f=$OUT/${L}_s${si}_r$rep
      EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -k 10 300 python3 bench.py ${SETS[$si]} > $f.json 2> $f.err
      rc=$?; [ $rc = 0 ] || { echo "$L set $si rep $rep rc=$rc"; tail -3 $f.err; exit $rc; }
      python3 -c "import json; b=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]); print('$L', 'set$si', '%.4g' % b['value'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), [round(t*1e6,1) for t in b['times_s']][:5])"
    done
  done
done
