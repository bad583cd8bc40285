#!/bin/bash
# round 4: two-deep Gx prefetch in the forward recurrence: stamps, op tests, solo tool, headline
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_k
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "lstm" > $O/tests_ops.log 2>&1
rc=$?; echo "op tests rc=$rc"; tail -2 $O/tests_ops.log; [ $rc -eq 0 ] || exit $rc
H=128 STAMP_CFGS=1:0 timeout -k 10 300 python -u tools/tools_lstm_stamps.py > $O/stamps128_gx2.log 2>&1 || exit 1
H=256 STAMP_CFGS=1:0,1:2 timeout -k 10 300 python -u tools/tools_lstm_stamps.py > $O/stamps256_gx2.log 2>&1 || exit 1
grep -E "^fwd|^bwd" $O/stamps128_gx2.log $O/stamps256_gx2.log
timeout -k 10 300 python -u tools/tools_lstm_solo.py > $O/solo_gx2.log 2>&1 || exit 1
grep -v amdgpu $O/solo_gx2.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --secondary 0 --cpu-baseline 0 --steps 30 > $O/bench.$i.log 2>&1 || exit 1
  echo "bench $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench.$i.log | head -1)"
done
