#!/bin/bash
# Round-2 GPU session: parity tests, smoke, the driver's bench commands, and a
# 2-rank torchrun rehearsal of the N>1 path (both ranks on device 0, gloo).
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "GPU step '$2' ended with $1: stopping"; exit $1;; esac; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${T_TEST:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; grep -E 'passed|failed|error' $OUT/pytest_gpu.log | tail -5; fatal $rc pytest
  timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; fatal $rc smoke
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err
rc=$?; echo "bench(20/5) rc=$rc"; cat $OUT/bench_s20.json; tail -3 $OUT/bench_s20.err; fatal $rc bench20
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err; fatal $rc bench
if [ "${TORCHRUN:-1}" = 1 ]; then
  EMCMC_BENCH_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_n2.json 2> $OUT/bench_n2.err
  rc=$?; echo "torchrun rc=$rc"; cat $OUT/bench_n2.json; tail -3 $OUT/bench_n2.err; fatal $rc torchrun
fi
if [ "${PROFILE:-0}" = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
  find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \; | head -20
fi
