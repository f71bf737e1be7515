#!/bin/bash
# Round-4 session 9: the driver's 20-step window with and without per-launch
# dispatch events (interleaved), and cfg 4 / cfg 3 on the tiled layout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_s9; mkdir -p $OUT
for rep in 1 2 3; do
  for T in "" "--no-kernel-timing"; do
    f=$OUT/s20${T:+_noev}_r$rep
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu $T > $f.json 2> $f.err || { echo "rc=$? $f"; tail -3 $f.err; exit 1; }
    python3 -c "import json; b=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]); print('s20 $T', '%.4g' % b['value'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), [round(t*1e6,1) for t in b['times_s']][:5])"
  done
done
for W in cfg4 cfg3; do
  f=$OUT/bench_$W
  timeout -k 10 600 python3 bench.py --workload $W --no-cpu > $f.json 2> $f.err || { echo "rc=$? $f"; tail -3 $f.err; exit 1; }
  python3 -c "import json; b=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]); print('$W', '%.4g' % b['value'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), b.get('parity'))"
done
