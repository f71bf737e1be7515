#!/bin/bash
# Round-4 session 13: the run-time chol kernel with one shared substitution sweep for
# ltd and the likelihood at D ≥ 40 — its GPU tests, then D = 40…64 in both likelihood
# modes against the three-sweep build (EMCMC_RTC_EXTRA=-DEMCMC_CHOL_SHARED=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_s13; mkdir -p $OUT gpurun_out/rtc_cache
trap 'cp -n extensiblemcmc.jl_amd/lib/rtc_cache/*.co gpurun_out/rtc_cache/ 2>/dev/null; true' EXIT
echo "== pytest chol $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_chol.py -m gpu -x -q --timeout 900 --timeout-method thread > $OUT/pytest_chol.txt 2>&1 || { tail -30 $OUT/pytest_chol.txt; exit 1; }
tail -1 $OUT/pytest_chol.txt
for LLM in per_obs suffstat; do
  for X in "" "-DEMCMC_CHOL_SHARED=0"; do
    tag=${LLM}${X:+_threesweep}
    echo "== $tag $(date +%T)"
    EMCMC_RTC_EXTRA="$X" timeout -k 10 900 python3 scripts/bench_dense.py --dims 40,48,56,64 --ll $LLM --general 0 > $OUT/dense_$tag.jsonl 2> $OUT/dense_$tag.err || { echo rc=$?; tail -3 $OUT/dense_$tag.err; exit 1; }
    python3 -c "
import json
for l in open('$OUT/dense_$tag.jsonl'):
    r=json.loads(l); print('$tag', r['D'], '%.3g' % r['chain_steps_per_s'])"
  done
done
