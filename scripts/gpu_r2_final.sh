#!/bin/bash
# Round-2 closing GPU session: full -m gpu suite + smoke + cfg 2 bench lines (gpu_r2.sh),
# interleaved cfg 4 A/B against the previous library, cfg 4 bench and its rocprofv3 kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "GPU step '$2' ended with $1: stopping"; exit $1;; esac; }
PROFILE=0 TORCHRUN=0 bash scripts/gpu_r2.sh; rc=$?; [ $rc = 0 ] || exit $rc
LIBS="${ABLIBS:-libemcmc_base libemcmc libemcmc_base libemcmc libemcmc_base libemcmc}" bash scripts/ab_cfg4.sh; rc=$?; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload cfg4 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
rc=$?; echo "bench cfg4 rc=$rc"; cut -c1-400 $OUT/bench_cfg4.json; tail -3 $OUT/bench_cfg4.err; fatal $rc bench_cfg4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg4 -o run -- python3 bench.py --workload cfg4 --no-cpu --steps 400 > $OUT/prof_cfg4.log 2>&1
rc=$?; echo "rocprof cfg4 rc=$rc"; fatal $rc rocprof_cfg4
find $OUT/prof_cfg4 -name '*kernel_stats.csv' -exec cut -d, -f1-4 {} \;
