#!/bin/bash
# round 4: fused integrator on the T = 1 generation frames
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_o
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_models.py \
  -k "generation or q9 or prediction or sampling" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  MRG_FUSED_T1=$v timeout -k 10 600 python -u tools/tools_bench_models.py 3 gen 1 > $O/gen_t1_$v.log 2>&1 || { echo "gen failed"; tail -5 $O/gen_t1_$v.log; exit 1; }
  echo "fused_t1=$v: $(grep -o '"ms_per_clip_batch": [0-9.]*' $O/gen_t1_$v.log | tail -1)"
done
