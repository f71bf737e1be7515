#!/bin/bash
# Round 3 end: the GPU test suite, smoke(), the driver's exact bench command, the
# 1000-step default and cfg 4, each under its own limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RTAG:-r3final}
mkdir -p $OUT
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 ${T_STEP:-600} "$@"
  local rc=$?
  echo "rc=$rc"
  case $rc in 0) ;; *) echo "GPU step $name ended with $rc: stopping"; exit $rc;; esac
}
step pytest python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
tail -3 $OUT/pytest_gpu.txt
step smoke python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
step bench_driver python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err
step bench_default python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
step bench_cfg4 python3 bench.py --workload cfg4 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
for f in bench_s20 bench bench_cfg4; do
  python3 -c "import json; b=json.loads([l for l in open('$OUT/$f.json') if l.startswith('{')][-1]); print('$f', '%.4g' % b['value'], 'frac %.3f' % b['roofline']['frac'], 'kernel %.4g' % b['kernel_chain_steps_per_s'])"
done
