#!/bin/bash
# Interleaved A/B of the cfg 4 launch group for the libraries named in LIBS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ab_cfg4; mkdir -p $OUT
for L in ${LIBS:-libemcmc libemcmc}; do
  EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -k 10 200 python bench.py --workload cfg4 --no-cpu --steps ${STEPS:-400} --warmup 20 > $OUT/$L.json 2> $OUT/$L.err
  rc=$?; echo "$L rc=$rc"; python3 -c "import json,sys; d=json.loads(open('$OUT/$L.json').read().strip().splitlines()[-1]); print('$L', d['value'], d['kernel_chain_steps_per_s'])"; [ $rc = 0 ] || exit $rc
done
if [ -n "${TESTLIB:-}" ]; then
  EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$TESTLIB.so timeout -k 10 400 python -u -m pytest tests/test_gpu_mix.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_mix.log 2>&1
  rc=$?; echo "pytest mix ($TESTLIB) rc=$rc"; tail -3 $OUT/pytest_mix.log; exit $rc
fi
