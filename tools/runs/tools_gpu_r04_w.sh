#!/bin/bash
# round 4: GRU config with weight gradients deferred beside the GRU recurrences; parity + A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_w
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py \
  tests/test_gpu_capture.py -k "gru or replayed_step" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  MRG_WGRAD_DEFER=$v timeout -k 10 300 python -u tools/tools_bench_models.py 5 gru 1 > $O/gru_defer$v.log 2>&1 || exit 1
  echo "defer=$v: $(grep -o '{.*' $O/gru_defer$v.log | tail -1)"
done
