#!/bin/bash
# LSTM tuning round-trip: LSTM parity tests, phase stamps, then bench at each group size.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "lstm or LSTM" -p no:cacheprovider > gpurun_out/lstm_tests.log 2>&1 || { echo "lstm tests failed"; tail -30 gpurun_out/lstm_tests.log; exit 1; }
tail -2 gpurun_out/lstm_tests.log
timeout -k 10 300 python tools_lstm_stamps.py > gpurun_out/stamps.log 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps.log
for g in ${BENCH_GROUPS:-8}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --lstm-group $g > gpurun_out/bench_g$g.log 2>&1 || { echo "bench g$g failed"; tail -20 gpurun_out/bench_g$g.log; exit 1; }
  echo "g=$g"; tail -1 gpurun_out/bench_g$g.log | cut -c1-400
done
