#!/bin/bash
# Round-4 session 10: tiled (default) vs untiled (EMCMC_SOA_TILE=0, every unit and the
# run-time kernels) on cfg 2 (20 and 1000 steps), cfg 4 and the general-kernel lines;
# then the 20-step window with and without dispatch events.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_s10; mkdir -p $OUT gpurun_out/rtc_cache
trap 'cp -n extensiblemcmc.jl_amd/lib/rtc_cache/*.co gpurun_out/rtc_cache/ 2>/dev/null; true' EXIT
for rep in 1 2; do
  for L in libemcmc libemcmc_untiled; do
    for S in "--steps 20 --warmup 5" "--steps 1000 --warmup 100" "--workload cfg4"; do
      f=$OUT/${L}_$(echo $S | tr -d ' -')_r$rep
      EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -k 10 300 python3 bench.py $S --no-cpu > $f.json 2> $f.err || { echo "rc=$? $f"; tail -3 $f.err; exit 1; }
      python3 -c "import json; b=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]); print('$L', '$S', '%.4g' % b['value'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), b.get('parity', {}).get('final_theta_ll_bitwise'))"
    done
    f=$OUT/${L}_general_r$rep
    EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -k 10 900 python3 scripts/bench_general.py --only haario_dense_d32,haario_dense_d32_general,mala_gsn_d32,pcn_user_d32 > $f.jsonl 2> $f.err || { echo "rc=$? $f"; tail -3 $f.err; exit 1; }
    python3 -c "
import json
for l in open('$f.jsonl'):
    r=json.loads(l); print('$L', r['workload'], '%.4g' % r['update_steps_per_s'])"
  done
done
for rep in 1 2 3; do
  for T in "" "--no-kernel-timing"; do
    f=$OUT/s20${T:+_noev}_r$rep
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu $T > $f.json 2> $f.err || { echo "rc=$? $f"; tail -3 $f.err; exit 1; }
    python3 -c "import json; b=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]); print('s20 $T', '%.4g' % b['value'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), [round(t*1e6,1) for t in b['times_s']][:5])"
  done
done
