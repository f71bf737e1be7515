#!/bin/bash
# MALA GPU parity tests, then cfg3 bench lines for each library in LIBS (same box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/mala; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_mala.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest mala rc=$rc"; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
for L in ${LIBS:-libemcmc}; do
  EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -k 10 300 python bench.py --workload cfg3 --no-cpu --steps ${STEPS:-60} --warmup 5 > $OUT/$L.json 2> $OUT/$L.err
  rc=$?; echo "$L rc=$rc $(python -c "import json;d=json.load(open('$OUT/$L.json'));print(d['value'], d['roofline']['achieved'], d['roofline']['avg_launch_ms'])")"
  [ $rc = 0 ] || exit $rc
done
