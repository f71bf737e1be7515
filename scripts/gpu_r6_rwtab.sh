#!/bin/bash
# r6: the schedule kernel with its update tables through one base pointer — bench lines of the
# rw_block shapes (one process each) and the block parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6_rwtab}
mkdir -p "$OUT"
mkdir -m 700 -p gpurun_out/rtc_cache_${TAG:-r6_rwtab} && cp -p extensiblemcmc.jl_amd/lib/rtc_cache/*.co gpurun_out/rtc_cache_${TAG:-r6_rwtab}/
export EMCMC_RTC_CACHE=$PWD/gpurun_out/rtc_cache_${TAG:-r6_rwtab}
W=mwg_d32_two_blocks,mwg_d64_two_blocks,rw_product_normal_d32,rw_standard_mvnormal_d32,unif_pos_d32
for r in 1 2; do
  echo "== lines $r $(date +%T)"
  timeout -k 10 300 python3 -u scripts/bench_general.py --only $W > "$OUT/lines_$r.jsonl" 2> "$OUT/lines_$r.err"
  rc=$?; echo "rc=$rc"; [ $rc = 0 ] || { tail -5 "$OUT/lines_$r.err"; exit $rc; }
  python3 -c "
import json
for l in open('$OUT/lines_$r.jsonl'):
    d=json.loads(l); print(d['workload'], '%.3e'%d['update_steps_per_s'])"
done
echo "== parity $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_rwblock.py tests/test_gpu_priors.py tests/test_gpu_mwg.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?; echo "rc=$rc"; tail -3 "$OUT/pytest.txt"
exit $rc
