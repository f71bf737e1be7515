#!/bin/bash
# r6 final A: full GPU suite, smoke and every bench_general workload (one process each), with
# every run-time kernel captured into a private cache dir seeded from lib/rtc_cache (entries this
# session never reads are listed in unused.txt, by access time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp EMCMC_RTC_LOG=1
TAG=${TAG:-r6_finalA}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
CAP=gpurun_out/rtc_cache_$TAG
mkdir -m 700 -p "$CAP" && cp -p extensiblemcmc.jl_amd/lib/rtc_cache/*.co "$CAP"/ && chmod 600 "$CAP"/*.co
touch -a -m -d '2020-01-01' "$CAP"/*.co
export EMCMC_RTC_CACHE=$PWD/$CAP
(while true; do date +%T >> "$OUT/tick.txt"; sleep 30; done) &
TICK=$!
trap 'kill $TICK 2>/dev/null; true' EXIT
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?; echo "rc=$rc"; tail -3 "$OUT/$name.txt" | cut -c1-240
  [ $rc = 0 ] || exit $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_general 600 python3 -u scripts/bench_general.py
find "$CAP" -name '*.co' -atime +1000 -printf '%f\n' > "$OUT/unused.txt"; wc -l < "$OUT/unused.txt"
