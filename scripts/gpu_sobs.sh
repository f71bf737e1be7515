#!/bin/bash
# Scalar-observation variant session: parity tests, then interleaved A/B of the
# headline kernel (LPC=2 LDS observations vs one lane per chain, SGPR observations).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "GPU step '$2' ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chol.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_sobs.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'passed|failed|Error|error' $OUT/pytest_sobs.log | tail -8; fatal $rc pytest
[ $rc = 0 ] || exit $rc
timeout -k 10 400 python scripts/kbench.py --grid "${GRID:-2:0,1:4,1:0}" --hist full --ll per_obs,suffstat --rounds 3 --steps 400 > $OUT/kbench_sobs.json 2> $OUT/kbench_sobs.err
rc=$?; echo "kbench rc=$rc"; cat $OUT/kbench_sobs.json; tail -3 $OUT/kbench_sobs.err; fatal $rc kbench
