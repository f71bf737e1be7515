#!/bin/bash
# cfg4 session: mix GPU tests, cfg4 bench, rocprofv3 kernel trace of the cfg4 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "GPU step '$2' ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_mix.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_mix.log 2>&1
rc=$?; echo "pytest mix rc=$rc"; tail -4 $OUT/pytest_mix.log; fatal $rc pytest; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload cfg4 ${BENCH_ARGS:-} > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_cfg4.json; tail -3 $OUT/bench_cfg4.err; fatal $rc bench
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg4 -o run -- python3 bench.py --workload cfg4 --no-cpu --steps 400 ${BENCH_ARGS:-} > $OUT/prof_cfg4.log 2>&1
rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
find $OUT/prof_cfg4 -name '*kernel_stats.csv' -exec cat {} \;
