#!/bin/bash
# Round-4 session 14: MALA on the general kernel with the gradient carried between the
# steps of a launch — its GPU tests, then the general-kernel lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_s14; mkdir -p $OUT gpurun_out/rtc_cache
trap 'cp -n extensiblemcmc.jl_amd/lib/rtc_cache/*.co gpurun_out/rtc_cache/ 2>/dev/null; true' EXIT
echo "== pytest mala $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_mala_general.py tests/test_gpu_mala.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest_mala.txt 2>&1 || { tail -30 $OUT/pytest_mala.txt; exit 1; }
tail -1 $OUT/pytest_mala.txt
timeout -k 10 600 python3 scripts/bench_general.py --only mala_gsn_d32,pcn_user_d32 > $OUT/bench_general.jsonl 2> $OUT/bench_general.err || { echo rc=$?; tail -3 $OUT/bench_general.err; exit 1; }
cat $OUT/bench_general.jsonl
