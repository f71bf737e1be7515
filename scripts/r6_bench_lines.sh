#!/bin/bash
# Round-6 bench lines, each under its own limit (a failure ends the script):
# the driver's 20-step command, the 1000-step default, cfg 4, cfg 3, cfg 5's shard 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_bench}; mkdir -p $OUT
run() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 ${T_BENCH:-420} python3 -u bench.py "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err
  local rc=$?; echo "rc=$rc"; cut -c1-200 $OUT/bench_$name.json
  [ $rc = 0 ] || { tail -5 $OUT/bench_$name.err; exit $rc; }
}
run s20 --gpus 1 --steps 20 --warmup 5
run default
run cfg4 --workload cfg4
run cfg3 --workload cfg3
run cfg5_shard0 --workload cfg5 --shard 0
