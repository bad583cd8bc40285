#!/bin/bash
# GPU tests of the models + the other BASELINE configs' graph-replayed timings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 500 python tools/tools_bench_models.py 5 all 1 > gpurun_out/models_a.log 2>&1 || { tail -20 gpurun_out/models_a.log; exit 1; }
tail -1 gpurun_out/models_a.log
