#!/bin/bash
# Round-4 session 3: the MINW=2 diag kernels (inst_diag2.hip) — fused-kernel GPU
# parity tests, then an interleaved A/B against the uncapped build (--variant 128).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_minw2; mkdir -p $OUT
echo "== pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for rep in 1 2 3; do
  for V in 0 128; do
    for S in "--steps 20 --warmup 5" "--steps 1000 --warmup 100"; do
      f=$OUT/v${V}_$(echo $S | cut -d' ' -f2)_r$rep
      timeout -k 10 300 python3 bench.py --gpus 1 $S --no-cpu --variant $V > $f.json 2> $f.err || { echo "rc=$? $f"; tail -3 $f.err; exit 1; }
      python3 -c "import json; b=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]); print('v$V', '$S', '%.4g' % b['value'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), b['config']['kernel'], [round(t*1e6,1) for t in b['times_s']][:5], b.get('parity'))"
    done
  done
done
echo "== trace20 (MINW=2) $(date +%T)"
EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/libemcmc_trace.so timeout -k 10 180 python3 scripts/trace_diag.py --steps 20 --reps 3 > $OUT/trace20.jsonl 2> $OUT/trace20.err || { tail $OUT/trace20.err; exit 1; }
cut -c1-600 $OUT/trace20.jsonl
