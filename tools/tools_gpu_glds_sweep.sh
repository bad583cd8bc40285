#!/bin/bash
# LDS-DMA x6 GEMM: parity test, then per-shape timing for each ring depth / column tile (0 = old kernel).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "glds" -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/glds_tests.log 2>&1 || { echo "glds tests failed"; tail -30 gpurun_out/glds_tests.log; exit 1; }
tail -1 gpurun_out/glds_tests.log
for cfg in ${CFGS:-"0 128" "2 128" "3 128" "4 128" "2 64" "3 64"}; do
  set -- $cfg
  echo "== glds depth $1 bn $2"
  MRG_GEMM_GLDS=$1 MRG_GEMM_GLDS_BN=$2 timeout -k 10 90 python tools/tools_gemm_bench.py 1 > gpurun_out/glds_$1_$2.log 2>&1 || { echo "failed rc=$?"; tail -5 gpurun_out/glds_$1_$2.log; exit 1; }
  grep -E "Gx|fwd|NT" gpurun_out/glds_$1_$2.log
done
