#!/bin/bash
# Other BASELINE configs, graph-replayed, with weight gradients on the side stream (A) and on one
# stream (B, MRG_WGRAD_STREAM=0).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/tools_bench_models.py 5 all 1 > gpurun_out/models_a.log 2>&1 || { tail -20 gpurun_out/models_a.log; exit 1; }
tail -8 gpurun_out/models_a.log
MRG_WGRAD_STREAM=0 timeout -k 10 500 python tools/tools_bench_models.py 5 all 1 > gpurun_out/models_b.log 2>&1 || { tail -20 gpurun_out/models_b.log; exit 1; }
tail -8 gpurun_out/models_b.log
