#!/bin/bash
# Round-4 session 16: Engine.run host fast path (raw step address, memoised) — the GPU
# suite, then the driver's 20-step command and the default bench, 3 reps each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4_s16; mkdir -p $OUT
echo "== pytest gpu $(date +%T)"
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do
  for A in "--steps 20 --warmup 5" ""; do
    tag=$(echo "s${A:8:4}" | tr -d ' -'); f=$OUT/b${tag}_r$rep
    timeout -k 10 300 python3 bench.py $A --no-cpu > $f.json 2> $f.err || { echo "rc=$? $f"; tail -3 $f.err; exit 1; }
    python3 -c "import json; b=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]); print('$tag', '%.4g' % b['value'], 'ms/step %.4g' % b['ms_per_step'], 'kernel %.4g' % b.get('kernel_chain_steps_per_s', 0), b.get('parity', {}).get('final_theta_ll_bitwise'))"
  done
done
