#!/bin/bash
# round 4: kernel census of the GRU-config train step (graph replay)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_x
mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/gru -o run -- \
  python3 $R/tools/tools_bench_models.py 5 gru 1 > $O/gru.log 2>&1 || { echo "trace failed"; tail -5 $O/gru.log; exit 1; }
cp /tmp/gru/run_kernel_stats.csv $O/gru_stats.csv
grep -o '{.*' $O/gru.log | tail -1
