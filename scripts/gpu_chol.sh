#!/bin/bash
# Correlated-Σ kernel session: parity tests, general/dense throughput, rocprof kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "GPU step '$2' ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_chol.py tests/test_gpu_priors.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_chol.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'passed|failed|Error|error' $OUT/pytest_chol.log | tail -8; fatal $rc pytest
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_general.py > $OUT/bench_general.json 2> $OUT/bench_general.err
rc=$?; echo "bench_general rc=$rc"; cat $OUT/bench_general.json; tail -3 $OUT/bench_general.err; fatal $rc bench_general
if [ "${PROFILE:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/genprof -o run -- python3 scripts/bench_general.py > $OUT/genprof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
  find $OUT/genprof -name '*kernel_stats.csv' -exec cat {} \;
fi
