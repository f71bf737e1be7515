#!/bin/bash
# Round-4 session 2: per-wave timeline of the cfg 2 launch (trace build), then an
# interleaved A/B of the tiled-history timing variant at 20 and 100 steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_trace; mkdir -p $OUT
echo "== trace20 $(date +%T)"
EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/libemcmc_trace.so timeout -k 10 180 python3 scripts/trace_diag.py --steps 20 > $OUT/trace20.jsonl 2> $OUT/trace20.err || { tail $OUT/trace20.err; exit 1; }
cat $OUT/trace20.jsonl
echo "== trace100 $(date +%T)"
EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/libemcmc_trace.so timeout -k 10 180 python3 scripts/trace_diag.py --steps 100 --reps 3 > $OUT/trace100.jsonl 2> $OUT/trace100.err || { tail $OUT/trace100.err; exit 1; }
cat $OUT/trace100.jsonl
RTAG=r4_tiled_ab LIBS="libemcmc libemcmc_tiled" REPS=3 \
  ARGSETS="--gpus 1 --steps 20 --warmup 5 --no-cpu --no-parity;--gpus 1 --steps 1000 --warmup 100 --no-cpu --no-parity" \
  bash scripts/lib_ab.sh
