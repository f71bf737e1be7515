#!/bin/bash
# Round-4 session 19: scalar-load chunk size of the run-time chol kernel
# (EMCMC_CHOL_CHUNK through EMCMC_RTC_EXTRA, from a library built with kCholChunk
# temporarily read from that macro; 16 is the committed value) at D = 48 and 64,
# per-observation, 65,536 chains; each variant compiles into its own scratch cache.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_s19; mkdir -p $OUT
(while true; do date +%T >> $OUT/tick.txt; sleep 30; done) &
TICK=$!
trap 'kill $TICK 2>/dev/null; true' EXIT
for CH in ${CHUNKS:-16 8 24}; do
  echo "== chunk $CH $(date +%T)"
  EMCMC_RTC_CACHE=/tmp/rtcc_$CH EMCMC_RTC_EXTRA="-DEMCMC_CHOL_CHUNK=$CH" timeout -k 10 900 python3 -u scripts/bench_dense.py --dims 48,64 --general 0 > $OUT/chunk$CH.jsonl 2> $OUT/chunk$CH.err
  rc=$?; cat $OUT/chunk$CH.jsonl; [ $rc = 0 ] || { echo "rc=$rc"; tail -5 $OUT/chunk$CH.err; exit $rc; }
done
