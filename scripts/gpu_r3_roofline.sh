#!/bin/bash
# Round 3: the bench line's roofline made reproducible from profiles/.
#  1. the driver's exact command (bench.py --gpus 1 --steps 20 --warmup 5) under
#     rocprofv3: kernel trace, FETCH_SIZE, WRITE_SIZE, and a clock pass
#     (GRBM_GUI_ACTIVE / 8 / duration, MI355X_MICROARCH.md "DVFS give-back");
#  2. the same four passes on the 1000-step default;
#  3. the 20- vs 100-step gap: 1000 steps in 20-step launches, 1000 steps with a
#     100-iteration history ring, 20 timed steps after a 1000-step warm-up, 20
#     steps in one 20-step launch after a 5-step warm-up.
# Every GPU step has its own limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RTAG:-r3roof}
mkdir -p $OUT
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 ${T_STEP:-300} "$@"
  local rc=$?
  echo "rc=$rc"
  case $rc in 0) ;; 124|134|137|139) echo "GPU step $name ended with $rc: stopping"; exit $rc;; *) exit $rc;; esac
}
CLK="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for cfg in s20 s1000; do
  if [ $cfg = s20 ]; then B="--gpus 1 --steps 20 --warmup 5"; else B="--gpus 1"; fi
  mkdir -p $OUT/$cfg
  # the trace pass runs the command exactly as the driver does (CPU baseline included)
  step ${cfg}_trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$cfg/trace -o run -- \
    python3 bench.py $B > $OUT/$cfg/trace.json 2> $OUT/$cfg/trace.err
  step ${cfg}_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$cfg/fetch -o run -- \
    python3 bench.py $B --no-cpu > $OUT/$cfg/fetch.json 2> $OUT/$cfg/fetch.err
  step ${cfg}_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$cfg/write -o run -- \
    python3 bench.py $B --no-cpu > $OUT/$cfg/write.json 2> $OUT/$cfg/write.err
  step ${cfg}_clock rocprofv3 --pmc $CLK --output-format csv -d $OUT/$cfg/clock -o run -- \
    python3 bench.py $B --no-cpu > $OUT/$cfg/clock.json 2> $OUT/$cfg/clock.err
done
# the gap experiments (un-profiled; HIP-event kernel times in each line); GAP=0 skips them
if [ "${GAP:-1}" = 1 ]; then
step gap_spl20 python3 bench.py --no-cpu --steps 1000 --steps-per-launch 20 > $OUT/gap_spl20.json 2> $OUT/gap.err
step gap_ring100 python3 bench.py --no-cpu --steps 1000 --history-ring 100 > $OUT/gap_ring100.json 2>> $OUT/gap.err
step gap_warm1000 python3 bench.py --no-cpu --steps 20 --warmup 1000 > $OUT/gap_warm1000.json 2>> $OUT/gap.err
step gap_s20_spl20 python3 bench.py --no-cpu --steps 20 --warmup 5 --steps-per-launch 20 > $OUT/gap_s20_spl20.json 2>> $OUT/gap.err
step gap_s20_again python3 bench.py --no-cpu --steps 20 --warmup 5 > $OUT/gap_s20_again.json 2>> $OUT/gap.err
step gap_s1000_again python3 bench.py --no-cpu > $OUT/gap_s1000_again.json 2>> $OUT/gap.err
fi
python3 scripts/r3_roofline_summary.py $OUT > $OUT/summary.json; cat $OUT/summary.json
