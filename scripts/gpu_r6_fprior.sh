#!/bin/bash
# r6: the fused diagonal step with a separable prior — parity tests, then the bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp EMCMC_RTC_LOG=1
OUT=gpurun_out/${TAG:-r6_fprior}
mkdir -p "$OUT"
CAP=gpurun_out/rtc_cache_${TAG:-r6_fprior}
mkdir -m 700 -p "$CAP" && cp -p extensiblemcmc.jl_amd/lib/rtc_cache/*.co "$CAP"/
export EMCMC_RTC_CACHE=$PWD/$CAP
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fprior.py tests/test_gpu_rwblock.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?; echo "rc=$rc"; tail -12 "$OUT/pytest.txt" | cut -c1-250
[ $rc = 0 ] || exit $rc
echo "== lines $(date +%T)"
timeout -k 10 300 python3 -u scripts/bench_general.py --only ${LINES:-rw_product_normal_d32,rw_product_normal_d32_block,unif_pos_d32,unif_pos_d32_block} > "$OUT/lines.jsonl" 2> "$OUT/lines.err"
rc=$?; echo "rc=$rc"; cut -c1-250 "$OUT/lines.jsonl"
exit $rc
