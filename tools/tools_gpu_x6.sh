set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/tools_gemm_bench.py 1,0 > gpurun_out/gemm_x6.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/gemm_x6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_tests.log
exit $rc
