#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "GPU step '$2' ended with $1: stopping"; exit $1;; esac; }

timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -5 $OUT/pytest_gpu.log; fatal $rc pytest
[ "${SKIP_SMOKE:-0}" = 1 ] || { timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; cat $OUT/smoke.log | tail -3; fatal $rc smoke; }
timeout -k 10 ${T_BENCH:-600} python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err; fatal $rc bench
if [ "${PROFILE:-1}" = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
  find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \; | head -20
fi
