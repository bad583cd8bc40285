#!/bin/bash
# GEMM tuning: parity tests of the GEMM users, then per-shape timing for each forced (BK, tile) pair.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "linear or ffn or lstm or attention" -p no:cacheprovider > gpurun_out/gemm_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
for c in ${CONFIGS:-32:auto}; do
  bk=${c%%:*}; t=${c##*:}
  export MRG_GEMM_BK=$bk  # (ignored unless a BK variant is instantiated)
  if [ "$t" = "auto" ]; then unset MRG_GEMM_TILE; else export MRG_GEMM_TILE=$t; fi
  echo "=== BK $bk tile $t"
  timeout -k 10 300 python tools/tools_gemm_bench.py > gpurun_out/gemm_bench_$bk_$t.log 2>&1 || { echo "gemm bench failed"; tail -20 gpurun_out/gemm_bench_$bk_$t.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/gemm_bench_$bk_$t.log
done
