cd $GRAFT_REPO_ROOT
for K in 100 250 500 1000; do
  timeout -k 10 200 python bench.py --no-cpu --steps-per-launch $K --reps 3 > gpurun_out/spl_$K.json 2>/dev/null
  echo "K=$K rc=$? $(python -c "import json;d=json.load(open('gpurun_out/spl_$K.json'));print(d['value'], d['roofline']['avg_launch_ms'], d['kernel_chain_steps_per_s'])")"
done
