#!/bin/bash
# Round-4 session 15: moments kernel with sibling pacing (libemcmc_mpace) — mix GPU
# tests, then cfg 4 interleaved against the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_s15; mkdir -p $OUT
echo "== pytest mix (mpace) $(date +%T)"
EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/libemcmc_mpace.so timeout -k 10 900 python -u -m pytest tests/test_gpu_mix.py tests/test_gpu_mix_chol.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest_mix.txt 2>&1 || { tail -30 $OUT/pytest_mix.txt; exit 1; }
tail -1 $OUT/pytest_mix.txt
for rep in 1 2 3; do
  for L in libemcmc libemcmc_mpace; do
    f=$OUT/${L}_cfg4_r$rep
    EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -k 10 300 python3 bench.py --workload cfg4 --no-cpu > $f.json 2> $f.err || { echo "rc=$? $f"; tail -3 $f.err; exit 1; }
    python3 -c "import json; b=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]); print('$L', '%.4g' % b['value'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), b.get('parity', {}).get('final_theta_ll_bitwise'))"
  done
done
mkdir -p $OUT/trace
for L in libemcmc libemcmc_mpace; do
  EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace/$L -o run -- python3 bench.py --workload cfg4 --no-cpu --no-parity > $OUT/trace/$L.json 2> $OUT/trace/$L.err || { echo "trace rc=$?"; exit 1; }
  find $OUT/trace/$L -name '*kernel_stats.csv' -exec head -3 {} \;
done
