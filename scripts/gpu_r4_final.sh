#!/bin/bash
# Round-4 end-of-session GPU run: the GPU suite and smoke(), then the roofline passes
# of the driver's command and the 1000-step default (kernel trace, FETCH_SIZE and
# WRITE_SIZE each in its own rocprofv3 run, clock), then cfg 4 and cfg 3 lines.
# Each GPU step under its own limit; a fault/abort/timeout ends the script.  The
# run-time code objects the box compiled are copied to gpurun_out/rtc_cache.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RTAG:-r4_final}
mkdir -p $OUT gpurun_out/rtc_cache
(while true; do date +%T >> $OUT/tick.txt; sleep 30; done) &
TICK=$!
trap 'kill $TICK 2>/dev/null; cp -n extensiblemcmc.jl_amd/lib/rtc_cache/*.co gpurun_out/rtc_cache/ 2>/dev/null; true' EXIT
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 ${T_STEP:-600} "$@"
  local rc=$?
  echo "rc=$rc"
  case $rc in 0) ;; *) echo "GPU step $name ended with $rc: stopping"; exit $rc;; esac
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  T_STEP=1000 step pytest python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
  grep -E "passed|failed" $OUT/pytest_gpu.txt | tail -1
  step smoke python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
  tail -1 $OUT/smoke.txt
fi
CLK="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for cfg in s20 s1000; do
  if [ $cfg = s20 ]; then B="--gpus 1 --steps 20 --warmup 5"; else B="--gpus 1"; fi
  mkdir -p $OUT/$cfg
  step ${cfg}_trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$cfg/trace -o run -- \
    python3 bench.py $B > $OUT/$cfg/trace.json 2> $OUT/$cfg/trace.err
  step ${cfg}_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$cfg/fetch -o run -- \
    python3 bench.py $B --no-cpu > $OUT/$cfg/fetch.json 2> $OUT/$cfg/fetch.err
  step ${cfg}_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$cfg/write -o run -- \
    python3 bench.py $B --no-cpu > $OUT/$cfg/write.json 2> $OUT/$cfg/write.err
  step ${cfg}_clock rocprofv3 --pmc $CLK --output-format csv -d $OUT/$cfg/clock -o run -- \
    python3 bench.py $B --no-cpu > $OUT/$cfg/clock.json 2> $OUT/$cfg/clock.err
done
for b in s20 default cfg4 cfg3; do
  case $b in
    s20) args="--gpus 1 --steps 20 --warmup 5";;
    default) args="";;
    cfg4) args="--workload cfg4";;
    cfg3) args="--workload cfg3";;
  esac
  step bench_$b python3 bench.py $args > $OUT/bench_$b.json 2> $OUT/bench_$b.err
  python3 -c "import json; b=json.loads([l for l in open('$OUT/bench_$b.json') if l.startswith('{')][-1]); print('$b', '%.4g' % b['value'], 'frac %.3f' % b['roofline']['frac'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), b.get('parity'))"
done
python3 scripts/r3_roofline_summary.py $OUT > $OUT/summary.json && python3 -c "
import json; s=json.load(open('$OUT/summary.json'))
for c in ('s20','s1000'):
    o=s.get(c,{}); print(c, {k: o.get('rocprof_trace',{}).get(k) for k in ('timed_avg_ns','frac','frac_vs_bench_line')}, o.get('pmc_traffic',{}).get('traffic_over_algorithmic'))"
