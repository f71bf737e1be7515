#!/bin/bash
# Round profile of the headline bench command:
#   1. rocprofv3 --kernel-trace --stats (per-kernel durations)
#   2. rocprofv3 --pmc FETCH_SIZE        (own pass)
#   3. rocprofv3 --pmc WRITE_SIZE        (own pass)
# then scripts/pmc_summary.py → gpurun_out/prof_<tag>/summary.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BARGS="--no-cpu --steps ${STEPS:-300} --warmup ${WARMUP:-100} ${BENCH_ARGS:-}"
step() { echo "== $1"; shift; timeout -k 10 400 "$@"; rc=$?; echo "rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
step trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $BARGS > $OUT/trace.log 2>&1
step fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $BARGS > $OUT/fetch.log 2>&1
step write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $BARGS > $OUT/write.log 2>&1
python3 scripts/pmc_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
