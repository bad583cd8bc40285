#!/bin/bash
# GEMM per-shape timings (tools_gemm_bench.py) + GPU tests + headline bench (no CPU baseline).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/tools_gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 || { tail -20 gpurun_out/gemm_bench.log; exit 1; }
grep -E "dX|fwd|Gx|step-weighted" gpurun_out/gemm_bench.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline 0 > gpurun_out/bench_a.log 2>&1 || exit 1
python -c "import json;d=json.loads(open('gpurun_out/bench_a.log').read().strip().splitlines()[-1]);print('A', d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['kernels'].items()})"
