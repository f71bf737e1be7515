#!/bin/bash
# Round-end artifacts: bench line of each workload (with its CPU baseline),
# then the rocprofv3 kernel trace + FETCH/WRITE PMC passes of each
# (scripts/profile_all.sh).  Every GPU step has its own time limit; a failure
# ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
for W in ${WORKLOADS:-cfg2 cfg4 cfg3}; do
  timeout -k 10 400 python bench.py --workload $W > $OUT/bench_$W.json 2> $OUT/bench_$W.err
  rc=$?; echo "bench $W rc=$rc"; cut -c1-300 $OUT/bench_$W.json; [ $rc = 0 ] || exit $rc
done
[ "${PROFILE:-1}" = 1 ] && WORKLOADS="${WORKLOADS:-cfg2 cfg4 cfg3}" bash scripts/profile_all.sh
