#!/bin/bash
# Round-4 session 6: sibling-paced MINW=2 diag kernel (512-thread blocks) — fused
# GPU parity tests, per-wave timelines, and an interleaved A/B against the unpaced
# MINW=2 build (libemcmc_nopace) and the uncapped kernel (--variant 128).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_pace; mkdir -p $OUT
echo "== pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for S in 20 100; do
  echo "== trace$S paced $(date +%T)"
  EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/libemcmc_trace.so timeout -k 10 180 python3 scripts/trace_diag.py --steps $S --reps 3 --dump $OUT/trace$S > $OUT/trace$S.jsonl 2> $OUT/trace$S.err || { tail $OUT/trace$S.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/trace$S.jsonl'):
    r=json.loads(l); print({k: r[k] for k in ('kernel','event_us','start_skew_us','step_us_p50','end_p10_p50_p90_us','end_max_by_xcc_us','waves_per_simd_hist','simd_end_p10_p50_p90_max_us')})"
done
for rep in 1 2 3; do
  for cfg in "libemcmc 0" "libemcmc_nopace 0" "libemcmc 128"; do
    set -- $cfg; L=$1; V=$2
    for S in "--steps 20 --warmup 5" "--steps 1000 --warmup 100"; do
      f=$OUT/${L}_v${V}_$(echo $S | cut -d' ' -f2)_r$rep
      EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -k 10 300 python3 bench.py --gpus 1 $S --no-cpu --variant $V > $f.json 2> $f.err || { echo "rc=$? $f"; tail -3 $f.err; exit 1; }
      python3 -c "import json; b=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]); print('$L v$V', '$S', '%.4g' % b['value'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), b['config']['kernel'], [round(t*1e6,1) for t in b['times_s']][:5], b.get('parity', {}).get('final_theta_ll_bitwise'))"
    done
  done
done
