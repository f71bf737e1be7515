#!/bin/bash
# Round 3: cfg 3 and cfg 4 under rocprofv3 (kernel trace of the bench command with
# its CPU baseline), and cfg 4's compute counters (fp64 VALU instructions, VALU
# active cycles, clock) for the compute roofline on its line.  Every GPU step has
# its own limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RTAG:-r3cfgs}
mkdir -p $OUT
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 ${T_STEP:-300} "$@"
  local rc=$?
  echo "rc=$rc"
  case $rc in 0) ;; 124|134|137|139) echo "GPU step $name ended with $rc: stopping"; exit $rc;; *) exit $rc;; esac
}
timeout -k 5 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for w in cfg3 cfg4; do
  mkdir -p $OUT/$w
  step ${w}_trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$w/trace -o run -- \
    python3 bench.py --workload $w > $OUT/$w/trace.json 2> $OUT/$w/trace.err
done
F64="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
step cfg4_valu rocprofv3 --pmc $F64 --output-format csv -d $OUT/cfg4/valu -o run -- \
  python3 bench.py --workload cfg4 --no-cpu --steps 200 --warmup 100 > $OUT/cfg4/valu.json 2> $OUT/cfg4/valu.err
