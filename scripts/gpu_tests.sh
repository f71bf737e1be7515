#!/bin/bash
# Selected GPU tests (TESTS, default the whole -m gpu suite) and smoke(), each under
# its own limit; a progress file under gpurun_out/ ticks while hiprtc compiles run.
# A failure, timeout or abort ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RTAG:-tests}
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
step pytest python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout ${T_TEST:-600} --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
tail -3 $OUT/pytest_gpu.txt
if [ "${SMOKE:-1}" = 1 ]; then
  step smoke python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
  tail -1 $OUT/smoke.txt
fi
