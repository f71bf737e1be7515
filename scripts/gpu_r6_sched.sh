#!/bin/bash
# r6: MwG schedule lines (one process per workload) and their rocprofv3 kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6_sched
mkdir -p "$OUT"
W=mwg_d32_two_blocks,mwg_d32_two_blocks_wide,mwg_d64_two_blocks,mwg_d64_two_blocks_wide
echo "lines $(date +%T)"
timeout -k 10 400 python3 -u scripts/bench_general.py --only $W > "$OUT/bench_general_sched.jsonl" 2> "$OUT/lines_err.txt"
rc=$?; echo "rc=$rc"; cut -c1-200 "$OUT/bench_general_sched.jsonl"
[ $rc = 0 ] || exit $rc
echo "trace $(date +%T)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o sched -- python3 -u scripts/bench_general.py --inproc --only $W > "$OUT/traced.txt" 2>&1
rc=$?; echo "rc=$rc"; tail -4 "$OUT/traced.txt" | cut -c1-200
exit $rc
