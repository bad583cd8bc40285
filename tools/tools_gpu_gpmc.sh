#!/bin/bash
# bench (eager profile off) + SQ counters of the x6 GEMM on the LSTM input-projection shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log
bash tools/tools_gemm_pmc.sh
