#!/bin/bash
# One GPU session on the box (gpurun): every argument is a step NAME=COMMAND.  Each step
# runs under its own time limit (T_STEP seconds, default 900), its output goes to
# gpurun_out/$TAG/NAME.txt, a progress file ticks while it runs, and the first step that
# fails, aborts or times out ends the session (nothing else touches the GPU after it).
#   TAG=r5_s2 bash scripts/gpu_session.sh \
#     "tests=python -u -m pytest tests/test_gpu_block.py -m gpu -x -v --timeout 600 --timeout-method thread" \
#     "bench=python3 bench.py --steps 20 --warmup 5"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-session}
mkdir -p "$OUT"
(while true; do date +%T >> "$OUT/tick.txt"; sleep 30; done) &
TICK=$!
trap 'kill $TICK 2>/dev/null; true' EXIT
for spec in "$@"; do
  name=${spec%%=*}
  cmd=${spec#*=}
  echo "== $name $(date +%T): $cmd"
  timeout -k 10 "${T_STEP:-900}" bash -c "$cmd" > "$OUT/$name.txt" 2>&1
  rc=$?
  echo "rc=$rc"
  tail -n "${TAIL:-4}" "$OUT/$name.txt"
  if [ $rc != 0 ]; then
    echo "step $name ended with $rc: stopping"
    exit $rc
  fi
done
