#!/bin/bash
# rocprofv3 kernel stats of the graph-replayed C3 scheduled-sampling step (tools_bench_models.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${WHICH:-C3} -o run --output-format csv -- python3 $R/tools/tools_bench_models.py 2 ${WHICH:-C3} 1 > $R/gpurun_out/c3.log 2>&1 || { tail -5 $R/gpurun_out/c3.log; exit 1; }
rm -f $R/gpurun_out/${WHICH:-C3}/run_kernel_trace.csv; echo c3 ok
