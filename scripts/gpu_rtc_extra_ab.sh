#!/bin/bash
# Interleaved A/B of run-time-kernel build options (EMCMC_RTC_EXTRA) on bench_general workloads:
#   TAG=name W=workload,list ROUNDS=2 bash scripts/gpu_rtc_extra_ab.sh "" "-DFOO=1" ...
# (an empty argument is the default build); one process per workload and variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-rtc_ab}
mkdir -p "$OUT"
mkdir -m 700 -p "gpurun_out/rtc_cache_${TAG:-rtc_ab}" && cp -p extensiblemcmc.jl_amd/lib/rtc_cache/*.co "gpurun_out/rtc_cache_${TAG:-rtc_ab}/"
export EMCMC_RTC_CACHE=$PWD/gpurun_out/rtc_cache_${TAG:-rtc_ab}
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for X in "$@"; do
    i=$((i+1))
    echo "== v$i [$X] round $r $(date +%T)"
    EMCMC_RTC_EXTRA="$X" timeout -k 10 400 python3 -u scripts/bench_general.py --only "$W" > "$OUT/v${i}_r$r.jsonl" 2> "$OUT/v${i}_r$r.err"
    rc=$?; echo "rc=$rc"; [ $rc = 0 ] || { tail -5 "$OUT/v${i}_r$r.err"; exit $rc; }
    python3 -c "
import json
for l in open('$OUT/v${i}_r$r.jsonl'):
    d=json.loads(l); print('  ', d['workload'], '%.3e'%d['update_steps_per_s'], d['kernel'][:24])"
  done
done
