#!/bin/bash
# Full-status GPU session: parity tests, smoke, one bench line per workload.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "GPU step '$2' ended with $1: stopping"; exit $1;; esac; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${T_TEST:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -5 $OUT/pytest_gpu.log; fatal $rc pytest
  timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; fatal $rc smoke
fi
for wl in ${WORKLOADS:-cfg2 cfg4 cfg3}; do
  timeout -k 10 400 python bench.py --workload $wl ${BENCH_ARGS:-} > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err
  rc=$?; echo "bench $wl rc=$rc"; cat $OUT/bench_$wl.json; tail -3 $OUT/bench_$wl.err; fatal $rc bench_$wl
done
