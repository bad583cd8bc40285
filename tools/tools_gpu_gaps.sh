#!/bin/bash
# Kernel trace of the graph-replayed headline step (for idle-gap analysis: tools_gaps.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/gaps -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 --steps 5 --warmup 2 > $R/gpurun_out/gaps.log 2>&1 || { tail -5 $R/gpurun_out/gaps.log; exit 1; }
echo gaps ok
