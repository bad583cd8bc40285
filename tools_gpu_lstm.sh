#!/bin/bash
# LSTM tuning round-trip: phase stamps for both group sizes, then bench at each.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools_lstm_stamps.py > gpurun_out/stamps.log 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
for g in 16 8; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --lstm-group $g > gpurun_out/bench_g$g.log 2>&1 || { echo "bench g$g failed"; tail -20 gpurun_out/bench_g$g.log; exit 1; }
  echo "g=$g"; tail -1 gpurun_out/bench_g$g.log
done
