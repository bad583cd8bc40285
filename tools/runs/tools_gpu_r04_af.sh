#!/bin/bash
# round 4: VALU LSTM / GRU backward io waves stage and prefetch during the cell phase — recurrence
# parity tests, then headline and GRU-config A/B against the previous library (MRG_LIB_PATH), alternating
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_af
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -k "lstm or LSTM or gru or GRU or stack" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new base new base; do
  if [ $v = base ]; then export MRG_LIB_PATH=$R/multimodalreactiongeneration_amd/libmrg_base.so; else unset MRG_LIB_PATH; fi
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --secondary 0 > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$v.log; exit 1; }
  timeout -k 10 300 python3 tools/tools_bench_models.py 5 gru 1 > $O/gru_$v.log 2>&1 || { echo "gru failed"; tail -5 $O/gru_$v.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log | head -1) gru $(grep -o '"ms_per_step": [0-9.]*' $O/gru_$v.log | tail -1)"
done
