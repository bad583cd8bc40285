#!/bin/bash
# GEMM per-shape timing, then the PMC traffic passes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/tools_gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 || { echo "gemm bench failed"; tail -20 gpurun_out/gemm_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gemm_bench.log
if [ "${PMC:-1}" = "1" ]; then ./tools_pmc.sh; fi
