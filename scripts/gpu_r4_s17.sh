#!/bin/bash
# Round-4 session 17: carried-state loads issued before the table staging
# (EMCMC_EARLY_STATE=1, libemcmc_early) — diag GPU parity, the wave-timeline trace of
# both builds, then interleaved benches at 20 and 1000 steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_s17; mkdir -p $OUT
echo "== pytest parity (early) $(date +%T)"
EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/libemcmc_early.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_early.txt 2>&1 || { tail -30 $OUT/pytest_early.txt; exit 1; }
tail -1 $OUT/pytest_early.txt
for L in libemcmc_trace libemcmc_trace_early; do
  EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -k 10 300 python3 scripts/trace_diag.py --steps 20 > $OUT/${L}_20.jsonl 2> $OUT/${L}_20.err || { echo "trace rc=$?"; tail -5 $OUT/${L}_20.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/${L}_20.jsonl'):
    d=json.loads(l); print('$L', d['rep'], 'ev %.1f' % d['event_us'], 'stag', d['staging_us_p50'], 'state', d['state_us_p50'], d['state_us_max'], 'first', d['first_step_us_p50'], 'end', d['end_p10_p50_p90_us'], 'max', d['wave_span_us_max'])"
done
RTAG=r4_s17/ab LIBS="libemcmc libemcmc_early" REPS=3 ARGSETS="--gpus 1 --steps 20 --warmup 5 --no-cpu;--no-cpu" bash scripts/lib_ab.sh
