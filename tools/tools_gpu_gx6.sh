#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/tools_gemm_bench.py 1 > gpurun_out/gemm_x6.log 2>&1 || { tail -5 gpurun_out/gemm_x6.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gemm_x6.log
bash tools/tools_gemm_pmc.sh
