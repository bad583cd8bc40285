#!/bin/bash
# Secondary reference-rate bench (r = 8: 2400 audio frames per 300 prediction frames), no CPU baseline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --ratio 8 --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/bench_r8.log 2>&1 || { tail -20 gpurun_out/bench_r8.log; exit 1; }
tail -1 gpurun_out/bench_r8.log
