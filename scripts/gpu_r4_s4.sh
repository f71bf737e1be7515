#!/bin/bash
# Round-4 session 4: per-wave timelines of the MINW=2 and uncapped diag kernels,
# the MALA GPU tests with the division-free reciprocal, and an interleaved cfg 3
# A/B against the IEEE-division build (libemcmc_div, timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_s4; mkdir -p $OUT
for V in 0 128; do
  echo "== trace20 variant $V $(date +%T)"
  EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/libemcmc_trace.so timeout -k 10 180 python3 scripts/trace_diag.py --steps 20 --reps 3 --variant $V > $OUT/trace20_v$V.jsonl 2> $OUT/trace20_v$V.err || { tail $OUT/trace20_v$V.err; exit 1; }
  cut -c1-900 $OUT/trace20_v$V.jsonl
done
echo "== pytest mala $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_mala.py tests/test_gpu_mala_general.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest_mala.txt 2>&1 || { tail -30 $OUT/pytest_mala.txt; exit 1; }
tail -2 $OUT/pytest_mala.txt
RTAG=r4_s4/cfg3_ab LIBS="libemcmc libemcmc_div" REPS=3 ARGSETS="--workload cfg3 --steps 20 --warmup 2 --no-cpu --no-parity" bash scripts/lib_ab.sh
