#!/bin/bash
# Iteration session: GPU parity tests, kernel-variant sweep, optional PMC pass.
# Every GPU step runs under its own time limit; a fault/abort/timeout ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "GPU step '$2' ended with $1: stopping"; exit $1;; esac; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -5 $OUT/pytest_gpu.log; fatal $rc pytest
  [ $rc = 0 ] || exit $rc
fi
timeout -k 10 ${T_KB:-600} python scripts/kbench.py ${KB_ARGS:-} > $OUT/kbench.jsonl 2> $OUT/kbench.err
rc=$?; echo "kbench rc=$rc"; cat $OUT/kbench.jsonl; fatal $rc kbench
if [ -n "${PMC_ARGS:-}" ]; then
  VARIANT_ARGS="$PMC_ARGS" TAG=${PMC_TAG:-it} bash scripts/pmc.sh
fi
