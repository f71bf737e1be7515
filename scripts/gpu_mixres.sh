set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mix.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2c_mix.txt 2>&1 &&
timeout -k 10 200 python bench.py --workload cfg4 --steps 200 --warmup 20 --no-cpu > gpurun_out/r2c_cfg4_res.json 2> gpurun_out/r2c_cfg4_res.err &&
timeout -k 10 200 python bench.py --workload cfg4 --steps 200 --warmup 20 --no-cpu --variant 8 > gpurun_out/r2c_cfg4_stream.json 2> gpurun_out/r2c_cfg4_stream.err
