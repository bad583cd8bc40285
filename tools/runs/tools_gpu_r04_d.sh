#!/bin/bash
# round 4: warp-specialized weight-gradient kernel: bitwise test, then step A/B
set -o pipefail
O=gpurun_out/r04_d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_ops.py -k "specialized_kernel_bitwise or weight_grad_kernels or specialized_products" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/tools_wsp_bench.py > $O/wsp_bench.log 2>&1 || exit $?
cat $O/wsp_bench.log | grep -v amdgpu
for i in 1 2; do
  for v in 0 1 3; do
    MRG_GEMM_WSP=$v timeout -k 10 300 python -u bench.py --secondary 0 --cpu-baseline 0 --steps 30 > $O/bench_wsp$v.$i.log 2>&1 || exit $?
    echo "wsp=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_wsp$v.$i.log | head -1)"
  done
done
