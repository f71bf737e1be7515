#!/bin/bash
# Round-4 session 7: history-store A/B on the paced MINW=2 kernel — slot layout with
# nontemporal (default) or plain stores, 32-chain tiles nt / plain (timing only:
# the tiled builds' history readers are not adapted, so no parity replay).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_store_ab; mkdir -p $OUT
for rep in 1 2 3; do
  for L in libemcmc libemcmc_plain libemcmc_tiled libemcmc_tiledplain; do
    for S in "--steps 20 --warmup 5" "--steps 1000 --warmup 100"; do
      f=$OUT/${L}_$(echo $S | cut -d' ' -f2)_r$rep
      EMCMC_LIB=$PWD/extensiblemcmc.jl_amd/lib/$L.so timeout -k 10 300 python3 bench.py --gpus 1 $S --no-cpu --no-parity > $f.json 2> $f.err || { echo "rc=$? $f"; tail -3 $f.err; exit 1; }
      python3 -c "import json; b=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]); print('$L', '$S', '%.4g' % b['value'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), [round(t*1e6,1) for t in b['times_s']][:5])"
    done
  done
done
