#!/bin/bash
# Run-time compiled rwm_gsn_chol_kernel: its GPU tests, then the dense-Σ throughput
# A/B against the general kernel (scripts/bench_dense.py); each step under a limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RTAG:-dense}
mkdir -p $OUT
(while true; do date +%T >> $OUT/tick.txt; sleep 30; done) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 ${T_STEP:-900} "$@"
  local rc=$?
  echo "rc=$rc"
  case $rc in 0) ;; *) echo "GPU step $name ended with $rc: stopping"; exit $rc;; esac
}
step pytest python -u -m pytest tests/test_gpu_chol.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
tail -3 $OUT/pytest_gpu.txt
step bench_dense python3 -u scripts/bench_dense.py --dims ${DIMS:-12,20,40,48,64} > $OUT/bench_dense.jsonl 2> $OUT/bench_dense.err
cat $OUT/bench_dense.jsonl
