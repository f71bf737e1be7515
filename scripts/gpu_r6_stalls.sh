#!/bin/bash
# r6: where the schedule kernel's wave time goes (one PMC pass, 8 SQ counters) for the rw_block
# bench shapes, the cfg 2 step kernel alongside for reference
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6_stalls
mkdir -p "$OUT"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SMEM"
echo "== rw $(date +%T)"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/rw" -o run -- python3 -u scripts/bench_general.py --inproc --iters 50 --only mwg_d32_two_blocks,rw_product_normal_d32,rw_standard_mvnormal_d32,unif_pos_d32 > "$OUT/rw.txt" 2>&1
rc=$?; echo "rc=$rc"; [ $rc = 0 ] || { tail -5 "$OUT/rw.txt"; exit $rc; }
echo "== cfg2 $(date +%T)"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/cfg2" -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > "$OUT/cfg2.txt" 2>&1
rc=$?; echo "rc=$rc"; [ $rc = 0 ] || { tail -5 "$OUT/cfg2.txt"; exit $rc; }
