#!/bin/bash
# r6: full GPU suite + smoke with every run-time kernel captured into a private cache dir
# (seeded from lib/rtc_cache; entries this session never reads are listed in unused.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp EMCMC_RTC_LOG=1
OUT=gpurun_out/${TAG:-r6_suite}
mkdir -p "$OUT"
CAP=gpurun_out/rtc_cache_${TAG:-r6_suite}
mkdir -m 700 -p "$CAP" && cp -p extensiblemcmc.jl_amd/lib/rtc_cache/*.co "$CAP"/ && chmod 600 "$CAP"/*.co
touch -a -m -d '2020-01-01' "$CAP"/*.co
export EMCMC_RTC_CACHE=$PWD/$CAP
(while true; do date +%T >> "$OUT/tick.txt"; sleep 30; done) &
TICK=$!
trap 'kill $TICK 2>/dev/null; true' EXIT
echo "suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.txt" 2>&1
rc=$?; echo "rc=$rc"; tail -4 "$OUT/pytest_gpu.txt"
[ $rc = 0 ] || exit $rc
echo "smoke $(date +%T)"
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
rc=$?; echo "rc=$rc"; tail -3 "$OUT/smoke.txt"
find "$CAP" -name '*.co' -atime +1000 -printf '%f\n' > "$OUT/unused.txt"; wc -l < "$OUT/unused.txt"
exit $rc
