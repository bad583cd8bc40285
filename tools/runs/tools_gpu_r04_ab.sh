#!/bin/bash
# round 4: GRU defaults (4-member ring, io-wave backward) — GRU tests, GRU config step and census
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_ab
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -k "gru or GRU" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/tools_bench_models.py 5 gru 1 > $O/gru.log 2>&1 || { echo "bench failed"; tail -5 $O/gru.log; exit 1; }
grep -o '{.*' $O/gru.log | tail -1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/gru -o run -- \
  python3 $R/tools/tools_bench_models.py 5 gru 1 > $O/gru_prof.log 2>&1 || { echo "trace failed"; tail -5 $O/gru_prof.log; exit 1; }
cp /tmp/gru/run_kernel_stats.csv $O/gru_stats.csv
