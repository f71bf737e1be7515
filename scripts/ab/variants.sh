#!/bin/bash
# GPU tests, then the cfg2 kernel timed for each library named in LIBS
# (lib/libemcmc.so and timing/ablation builds next to it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/variants; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -5 $OUT/pytest_gpu.log; [ $rc = 0 ] || exit $rc
fi
for L in ${LIBS:-libemcmc}; do
  EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -k 10 300 python scripts/kbench.py --grid ${GRID:-2:0} --hist ${HIST:-full} --ll ${LL:-per_obs} --rounds 3 --steps 300 > $OUT/$L.json 2> $OUT/$L.err
  rc=$?; echo "$L rc=$rc"; cat $OUT/$L.json; [ $rc = 0 ] || exit $rc
done
