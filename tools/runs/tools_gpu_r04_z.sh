#!/bin/bash
# round 4: GRU ring of 4 vs 8 members at H = 256 — GRU parity tests with 4, then the GRU-config step each way
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_z
mkdir -p $O
cd $R
MRG_GRU_GROUP256=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -k "gru or GRU" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for g in 4 8 4 8; do
  MRG_GRU_GROUP256=$g timeout -k 10 300 python3 tools/tools_bench_models.py 5 gru 1 > $O/gru_$g.log 2>&1 || { echo "bench failed"; tail -5 $O/gru_$g.log; exit 1; }
  echo "G=$g $(grep -o '{.*' $O/gru_$g.log | tail -1)"
done
