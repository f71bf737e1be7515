#!/bin/bash
# The roofline evidence of the cfg 2 bench line (on the GPU box): for the driver's 20-step
# command and the 1000-step default, a rocprofv3 kernel trace and one PMC pass each for
# FETCH_SIZE, WRITE_SIZE and GRBM_GUI_ACTIVE (separate passes, MI355X_MICROARCH.md), then
# scripts/r3_roofline_summary.py → $OUT/summary.json.  Copy $OUT to profiles/<name> and run
# scripts/r3_traffic_table.py profiles/<name> to refresh profiles/pmc_traffic.json.
#   OUT=gpurun_out/r5_final bash scripts/roofline_profile.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/roofline}
for cfg in s20 s1000; do
  case $cfg in
    s20) B="--gpus 1 --steps 20 --warmup 5 --no-cpu" ;;
    s1000) B="--gpus 1 --no-cpu" ;;
  esac
  mkdir -p $OUT/$cfg
  for pass in trace fetch write clock; do
    case $pass in
      trace) P="--kernel-trace --stats" ;;
      fetch) P="--pmc FETCH_SIZE" ;;
      write) P="--pmc WRITE_SIZE" ;;
      clock) P="--pmc GRBM_GUI_ACTIVE" ;;
    esac
    echo "== $cfg $pass $(date +%T)"
    timeout -s KILL 300 rocprofv3 $P --output-format csv -d $OUT/$cfg/$pass -o run -- python3 bench.py $B \
      > $OUT/$cfg/$pass.json 2> $OUT/$cfg/$pass.err
    rc=$?; echo "rc=$rc"; [ $rc = 0 ] || { tail -5 $OUT/$cfg/$pass.err; exit $rc; }
  done
done
python3 scripts/r3_roofline_summary.py $OUT > $OUT/summary.json && head -c 1500 $OUT/summary.json
