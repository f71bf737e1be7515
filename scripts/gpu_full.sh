#!/bin/bash
# Full GPU test suite + smoke (round-end rehearsal).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "GPU step '$2' ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; grep -E 'passed|failed|Error' $OUT/pytest_gpu.log | tail -5; fatal $rc pytest
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; fatal $rc smoke
