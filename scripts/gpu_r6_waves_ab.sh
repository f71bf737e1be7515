#!/bin/bash
# r6 A/B: mwg_rw_block_kernel at 1 wave per SIMD (default) vs 2 (amdgpu_waves_per_eu(2), a few
# VGPRs spilled to scratch), interleaved twice, then the block parity tests at 2 waves.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6_waves_ab
mkdir -p "$OUT"
mkdir -m 700 -p gpurun_out/rtc_cache_waves && cp -p extensiblemcmc.jl_amd/lib/rtc_cache/*.co gpurun_out/rtc_cache_waves/
export EMCMC_RTC_CACHE=$PWD/gpurun_out/rtc_cache_waves
W=mwg_d32_two_blocks,rw_product_normal_d32,rw_standard_mvnormal_d32,unif_pos_d32
for r in 1 2; do
  for v in w1 w2; do
    if [ $v = w2 ]; then X="-DEMCMC_RW_WAVES_PER_EU=2"; A=1; else X=""; A=0; fi
    echo "== $v round $r $(date +%T)"
    EMCMC_RTC_EXTRA="$X" EMCMC_RW_ALLOW_SCRATCH=$A timeout -k 10 300 python3 -u scripts/bench_general.py --only $W > "$OUT/${v}_r$r.jsonl" 2> "$OUT/${v}_r$r.err"
    rc=$?; echo "rc=$rc"; [ $rc = 0 ] || { tail -5 "$OUT/${v}_r$r.err"; exit $rc; }
    python3 -c "
import json,sys
for l in open('$OUT/${v}_r$r.jsonl'):
    d=json.loads(l); print(d['workload'], '%.3e'%d['update_steps_per_s'])"
  done
done
echo "== parity at 2 waves $(date +%T)"
EMCMC_RTC_EXTRA="-DEMCMC_RW_WAVES_PER_EU=2" EMCMC_RW_ALLOW_SCRATCH=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_rwblock.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_w2.txt" 2>&1
rc=$?; echo "rc=$rc"; tail -3 "$OUT/pytest_w2.txt"
exit $rc
