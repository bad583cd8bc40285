#!/bin/bash
# LSTM tuning round-trip: LSTM parity tests, phase stamps, then bench, for each library variant in $LIBS.
set -o pipefail
mkdir -p gpurun_out
for L in ${LIBS:-libmrg.so}; do
  export MRG_LIB_PATH=$GRAFT_REPO_ROOT/multimodalreactiongeneration_amd/$L
  echo "=== $L"
  timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "lstm or LSTM" -p no:cacheprovider > gpurun_out/lstm_tests_$L.log 2>&1 || { echo "lstm tests failed"; tail -30 gpurun_out/lstm_tests_$L.log; exit 1; }
  tail -1 gpurun_out/lstm_tests_$L.log
  timeout -k 10 300 python tools/tools_lstm_stamps.py > gpurun_out/stamps_$L.log 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps_$L.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps_$L.log
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --secondary ${SECONDARY:-1} > gpurun_out/bench_$L.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$L.log; exit 1; }
  tail -1 gpurun_out/bench_$L.log | cut -c1-200
done
