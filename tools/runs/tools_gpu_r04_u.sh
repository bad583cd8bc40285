#!/bin/bash
# round 4: persistent GRU recurrence: parity tests, GRU-config step A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_u
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py \
  -k "gru" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error|assert" $O/tests.log | tail -14; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  MRG_GRU_PERSIST=$v timeout -k 10 400 python -u tools/tools_bench_models.py 3 gru 1 > $O/gru_$v.log 2>&1 || { tail -5 $O/gru_$v.log; exit 1; }
  echo "persist=$v: $(grep -o '{.*' $O/gru_$v.log | tail -1)"
done
