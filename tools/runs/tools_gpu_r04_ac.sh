#!/bin/bash
# round 4: LSTM forward ring of 4 (backward stays 8) at H = 256 — LSTM tests with it, then the headline each way
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_ac
mkdir -p $O
cd $R
MRG_LSTM_GROUP256_FWD=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "lstm or LSTM" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for g in 4 8 4 8; do
  MRG_LSTM_GROUP256_FWD=$g timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_$g.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$g.log; exit 1; }
  echo "Gfwd=$g $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$g.log | head -1)"
done
