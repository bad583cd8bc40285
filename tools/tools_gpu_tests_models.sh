set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 500 python tools/tools_bench_models.py 5 all 1 > gpurun_out/models_a.log 2>&1 || { tail -20 gpurun_out/models_a.log; exit 1; }
tail -1 gpurun_out/models_a.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline 0 > gpurun_out/bench_a.log 2>&1 || exit 1
python -c "import json;d=json.loads(open('gpurun_out/bench_a.log').read().strip().splitlines()[-1]);print('A', d['ms_per_step'])"
