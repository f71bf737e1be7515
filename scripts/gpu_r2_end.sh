#!/bin/bash
# Round-2 end-of-round GPU session: full -m gpu suite, smoke, cfg 2 bench lines,
# 2-rank torchrun rehearsal, cfg 2 rocprof kernel trace, cfg 4 bench + kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "GPU step '$2' ended with $1: stopping"; exit $1;; esac; }
PROFILE=${PROFILE:-1} bash scripts/gpu_r2.sh; rc=$?; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload cfg4 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
rc=$?; echo "bench cfg4 rc=$rc"; cat $OUT/bench_cfg4.json; tail -3 $OUT/bench_cfg4.err; fatal $rc bench_cfg4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg4 -o run -- python3 bench.py --workload cfg4 --no-cpu --steps 400 > $OUT/prof_cfg4.log 2>&1
rc=$?; echo "rocprof cfg4 rc=$rc"; fatal $rc rocprof_cfg4
find $OUT/prof_cfg4 -name '*kernel_stats.csv' -exec cat {} \;
