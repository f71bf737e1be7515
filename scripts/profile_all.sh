#!/bin/bash
# Round profiles of the three bench workloads (kernel trace + FETCH/WRITE PMC
# passes each), summarised into gpurun_out/prof_<tag>/summary.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for W in ${WORKLOADS:-cfg2 cfg4 cfg3}; do
  case $W in
    cfg2) T=r1 B="" S=1000 ;;
    cfg4) T=r1_cfg4 B="--workload cfg4" S=200 ;;
    cfg3) T=r1_cfg3 B="--workload cfg3" S=20; export WARMUP=5 ;;
  esac
  TAG=$T STEPS=$S BENCH_ARGS="$B" bash scripts/profile_round.sh > gpurun_out/profile_$W.log 2>&1
  rc=$?; echo "$W rc=$rc"; tail -3 gpurun_out/profile_$W.log; [ $rc = 0 ] || exit $rc
done
