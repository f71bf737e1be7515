#!/bin/bash
# Round 3 end (session 3): the whole GPU suite, smoke(), the driver's exact bench
# command, the 1000-step default, cfg 4, cfg 3, and a rocprofv3 kernel trace of the
# driver's command; each GPU step under its own limit, a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RTAG:-r3_end}
mkdir -p $OUT
(while true; do date +%T >> $OUT/tick.txt; sleep 30; done) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 ${T_STEP:-600} "$@"
  local rc=$?
  echo "rc=$rc"
  case $rc in 0) ;; *) echo "GPU step $name ended with $rc: stopping"; exit $rc;; esac
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
  grep -E "passed|failed" $OUT/pytest_gpu.txt | tail -1
  step smoke python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
  tail -1 $OUT/smoke.txt
fi
step bench_driver python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err
step bench_default python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
step bench_cfg4 python3 bench.py --workload cfg4 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
step bench_cfg3 python3 bench.py --workload cfg3 > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err
for f in bench_s20 bench bench_cfg4 bench_cfg3; do
  python3 -c "import json; b=json.loads([l for l in open('$OUT/$f.json') if l.startswith('{')][-1]); print('$f', '%.4g' % b['value'], 'frac %.3f' % b['roofline']['frac'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0))"
done
mkdir -p $OUT/s20
step s20_trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s20/trace -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20/trace.json 2> $OUT/s20/trace.err
find $OUT/s20/trace -name '*kernel_stats.csv' -exec head -5 {} \;
