#!/bin/bash
# Round-4 session 5: MALA GPU tests (division-free reciprocal), cfg 3 A/B against the
# IEEE-division build, and per-wave timelines of the MINW=2 kernel with placement.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_s5; mkdir -p $OUT
echo "== pytest mala $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_mala.py tests/test_gpu_mala_general.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest_mala.txt 2>&1 || { tail -30 $OUT/pytest_mala.txt; exit 1; }
tail -2 $OUT/pytest_mala.txt
for S in 20 100; do
  echo "== trace$S MINW=2 $(date +%T)"
  EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/libemcmc_trace.so timeout -k 10 180 python3 scripts/trace_diag.py --steps $S --reps 3 --dump $OUT/trace$S > $OUT/trace$S.jsonl 2> $OUT/trace$S.err || { tail $OUT/trace$S.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/trace$S.jsonl'):
    r=json.loads(l); print({k: r[k] for k in ('event_us','start_skew_us','step_us_p50','end_p10_p50_p90_us','end_p50_by_xcc_us','end_max_by_xcc_us','waves_per_simd_hist','cus_used','simd_end_p10_p50_p90_max_us')})"
done
RTAG=r4_s5/cfg3_ab LIBS="libemcmc libemcmc_div" REPS=3 ARGSETS="--workload cfg3 --steps 20 --warmup 2 --no-cpu --no-parity" bash scripts/lib_ab.sh
