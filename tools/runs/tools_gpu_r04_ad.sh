#!/bin/bash
# round 4: MFMA LSTM recurrences with io off the hand-off wait — LSTM / stack parity tests, then headline A/B against
# the previous library (libmrg_base.so, MRG_LIB_PATH) in alternating runs on one box
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_ad
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -k "lstm or LSTM or stack or mx" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new base new base; do
  if [ $v = base ]; then export MRG_LIB_PATH=$R/multimodalreactiongeneration_amd/libmrg_base.so; else unset MRG_LIB_PATH; fi
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --secondary 0 > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$v.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log | head -1)"
done
unset MRG_LIB_PATH
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/mxt -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
cp /tmp/mxt/run_kernel_stats.csv $O/stats.csv
