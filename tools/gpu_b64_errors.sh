set -e
mkdir -p gpurun_out/r05_h
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "plane_products" > gpurun_out/r05_h/ops.log 2>&1
for c in "MRG_WEIGHT_PLANES=0" "MRG_WEIGHT_PLANES=1" "MRG_GEMM_WIDE=0" "MRG_GEMM_WIDE=22" "MRG_GEMM_WIDE=13"; do
  env $c timeout -k 10 200 python -u tools/b64_errors.py 6 > gpurun_out/r05_h/err_$c.log 2>&1
done
