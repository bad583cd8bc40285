#!/bin/bash
# A/B: GPU tests, then the bench with the defaults (A) and with ${AB_ENV} / ${AB_ARGS} (B), no CPU baseline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/bench_a.log 2>&1 || { tail -20 gpurun_out/bench_a.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_a.log').read().strip().splitlines()[-1]);print('A', d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['kernels'].items()})"
env ${AB_ENV} timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 ${AB_ARGS} > gpurun_out/bench_b.log 2>&1 || { tail -20 gpurun_out/bench_b.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_b.log').read().strip().splitlines()[-1]);print('B', d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['kernels'].items()})"
