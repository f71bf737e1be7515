#!/bin/bash
# mix_chol_kernel session: its GPU tests with the other mix tests, the general-kernel
# workload lines of the round-3 verdict (scripts/bench_general.py), and a rocprofv3
# kernel trace of the fused correlated-Haario line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RTAG:-r4_mixchol}
mkdir -p $OUT gpurun_out/rtc_cache
trap 'cp -n extensiblemcmc.jl_amd/lib/rtc_cache/*.co gpurun_out/rtc_cache/ 2>/dev/null; true' EXIT
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 ${T_STEP:-600} "$@"
  local rc=$?
  echo "rc=$rc"
  case $rc in 0) ;; *) echo "GPU step $name ended with $rc: stopping"; exit $rc;; esac
}
step pytest python -u -m pytest ${TESTS:-tests/test_gpu_mix_chol.py tests/test_gpu_mix.py tests/test_gpu_mix_general.py} -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
grep -E "passed|failed" $OUT/pytest_gpu.txt | tail -1
step bench_general python3 scripts/bench_general.py --only ${ONLY:-haario_dense_d32,haario_dense_d32_general,mala_gsn_d32,pcn_user_d32} > $OUT/bench_general.jsonl 2> $OUT/bench_general.err
cat $OUT/bench_general.jsonl
mkdir -p $OUT/trace
step trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 scripts/bench_general.py --only haario_dense_d32 > $OUT/trace/line.json 2> $OUT/trace/err.txt
find $OUT/trace -name '*kernel_stats.csv' -exec head -6 {} \;
