#!/bin/bash
# Copy the round's bench lines and rocprofv3 summaries from gpurun_out/ (scratch,
# written by scripts/round_artifacts.sh on the GPU box) into profiles/ (tracked),
# and rebuild profiles/pmc_traffic.json, which bench.py reads for roofline.traffic.
set -e
cd "$(dirname "$0")/.."
R=${ROUND:-r1}
for pair in "cfg2:$R" "cfg4:${R}_cfg4" "cfg3:${R}_cfg3"; do
  W=${pair%%:*}; T=${pair#*:}; P=gpurun_out/prof_$T
  cp gpurun_out/bench_$W.json profiles/${T}_bench.json
  cp $P/trace/run_kernel_stats.csv profiles/${T}_kernel_stats.csv
  cp $P/fetch/run_counter_collection.csv profiles/${T}_pmc_fetch_size.csv
  cp $P/write/run_counter_collection.csv profiles/${T}_pmc_write_size.csv
  cp $P/summary.json profiles/${T}_summary.json
done
python3 - "$R" <<'PY'
import json, subprocess, sys
R = sys.argv[1]
out = {}
for tag, wl in ((R, "cfg2"), (R + "_cfg4", "cfg4")):
    b = json.load(open(f"profiles/{tag}_bench.json"))
    name, C, spl = b["roofline"]["kernel"], b["config"]["chains_per_gpu"], b["config"]["steps_per_launch"]
    r = subprocess.run(["python3", "scripts/make_traffic_json.py", f"profiles/{tag}_summary.json", name, str(C),
                        str(spl), tag], check=True, capture_output=True, text=True)
    d = json.loads(r.stdout)
    if wl == "cfg4":
        d[name]["note"] = ("per launch group: step kernel + mix_moments_kernel (+ mix_readjust_kernel every other "
                           "group at k=200), summed over the kernels of the timed run and divided by the step launches")
    out.update(d)
json.dump(out, open("profiles/pmc_traffic.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
