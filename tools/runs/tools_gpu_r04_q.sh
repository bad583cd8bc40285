#!/bin/bash
# round 4: bisect test_metaformer_benchmark_width_vs_oracle[1-4-300] over the schedule's switches
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_q
mkdir -p $O
cd $R
T="tests/test_gpu_models.py::test_metaformer_benchmark_width_vs_oracle"
for e in "X=0" "MRG_WGRAD_STREAM=0" "MRG_WGRAD_DEFER=0" "MRG_ENCODER_STACK=0" "MRG_FUSED_INTEGRATOR=0" "MRG_FORK_GUARD=0" "MRG_LSTM_SOLO=0" "MRG_LSTM_MX=0"; do
  env $e timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread "$T" > "$O/t_$e.log" 2>&1
  rc=$?
  echo "== $e rc=$rc: $(grep -E "passed|failed" "$O/t_$e.log" | tail -1)"
  grep -E "^E +AssertionError" "$O/t_$e.log" | head -2 | cut -c1-400
  [ $rc -le 1 ] || exit $rc
done
