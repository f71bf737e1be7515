#!/bin/bash
# Round-4 session 12: the run-time chol kernel at D = 40…64, per-observation and
# sufficient-statistic likelihood (where does the D ≥ 56 cliff come from?).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_s12; mkdir -p $OUT gpurun_out/rtc_cache
trap 'cp -n extensiblemcmc.jl_amd/lib/rtc_cache/*.co gpurun_out/rtc_cache/ 2>/dev/null; true' EXIT
for LLM in suffstat per_obs; do
  echo "== $LLM $(date +%T)"
  timeout -k 10 900 python3 scripts/bench_dense.py --dims 40,48,56,64 --ll $LLM --general 0 > $OUT/dense_$LLM.jsonl 2> $OUT/dense_$LLM.err || { echo rc=$?; tail -3 $OUT/dense_$LLM.err; exit 1; }
  cat $OUT/dense_$LLM.jsonl
done
