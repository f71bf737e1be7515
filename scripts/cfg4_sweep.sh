#!/bin/bash
# cfg 4 launch group timed at several chain counts (L_B footprint vs the 256 MB
# Infinity Cache), kernel trace per count.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/cfg4sweep; mkdir -p $OUT
for N in ${NS:-131072 65536 32768 16384}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/n$N -o run -- python3 bench.py --workload cfg4 --chains-per-gpu $N --steps 200 --warmup 0 --no-cpu --reps 1 > $OUT/n$N.json 2> $OUT/n$N.err
  rc=$?; echo "N=$N rc=$rc"; [ $rc = 0 ] || { tail -3 $OUT/n$N.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$OUT/n$N.json'));print('value',d['value'])"
  find $OUT/n$N -name '*kernel_stats.csv' -exec grep -E 'mix_' {} \;
done
