#!/bin/bash
# Round 4 GPU session driver: the GPU suite (or a subset: TESTS=...), smoke(), the
# driver's exact bench command, the 1000-step default, cfg 4, cfg 3 (BENCHES=...),
# a rocprofv3 kernel trace of the driver's command; each GPU step under its own
# limit, a failure ends the script.  The run-time code objects the box compiled are
# copied to gpurun_out/rtc_cache (harvested into lib/rtc_cache for the next runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RTAG:-r4}
mkdir -p $OUT gpurun_out/rtc_cache
(while true; do date +%T >> $OUT/tick.txt; sleep 30; done) &
TICK=$!
harvest() {
  kill $TICK 2>/dev/null
  cp -n extensiblemcmc.jl_amd/lib/rtc_cache/*.co gpurun_out/rtc_cache/ 2>/dev/null
  true
}
trap harvest EXIT
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 ${T_STEP:-600} "$@"
  local rc=$?
  echo "rc=$rc"
  case $rc in 0) ;; *) echo "GPU step $name ended with $rc: stopping"; exit $rc;; esac
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
  grep -E "passed|failed" $OUT/pytest_gpu.txt | tail -1
  step smoke python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
  tail -1 $OUT/smoke.txt
fi
for b in ${BENCHES:-s20 default cfg4 cfg3}; do
  case $b in
    s20) args="--gpus 1 --steps 20 --warmup 5";;
    default) args="";;
    cfg4) args="--workload cfg4";;
    cfg3) args="--workload cfg3";;
    *) args="$b";;
  esac
  step bench_$b python3 bench.py $args > $OUT/bench_$b.json 2> $OUT/bench_$b.err
  python3 -c "import json; b=json.loads([l for l in open('$OUT/bench_$b.json') if l.startswith('{')][-1]); print('$b', '%.4g' % b['value'], 'frac %.3f' % b['roofline']['frac'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), b.get('parity'))"
done
if [ "${TRACE:-1}" = 1 ]; then
  mkdir -p $OUT/s20
  step s20_trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s20/trace -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20/trace.json 2> $OUT/s20/trace.err
  find $OUT/s20/trace -name '*kernel_stats.csv' -exec head -5 {} \;
fi
