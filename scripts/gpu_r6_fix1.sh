#!/bin/bash
# r6: verify the engine-sequence fix (AOT code objects loaded at the first handle, run-time
# modules kept for the process), then the full GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp EMCMC_RTC_LOG=1
OUT=gpurun_out/r6_fix1
mkdir -p "$OUT"
# capture every run-time kernel this session compiles (copied into lib/rtc_cache afterwards)
mkdir -m 700 -p gpurun_out/rtc_cache_r6b && export EMCMC_RTC_CACHE=$PWD/gpurun_out/rtc_cache_r6b
(while true; do date +%T >> "$OUT/tick.txt"; sleep 30; done) &
TICK=$!
trap 'kill $TICK 2>/dev/null; true' EXIT
echo "seq $(date +%T)"
timeout -k 10 150 python3 -u scripts/bench_general.py --inproc --only mwg_d32_two_blocks,mwg_d32_two_blocks_wide,mwg_d64_two_blocks,mwg_d64_two_blocks_wide > "$OUT/seq.txt" 2>&1
rc=$?; echo "rc=$rc"; cut -c1-260 "$OUT/seq.txt" | tail -6
[ $rc = 0 ] || exit $rc
echo "suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.txt" 2>&1
rc=$?; echo "rc=$rc"; tail -4 "$OUT/pytest_gpu.txt"
exit $rc
