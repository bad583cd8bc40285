#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c2
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/tools/tools_c2_prof.py > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
cat $O/c2.log | grep C2
cd $R
python3 tools/tools_timeline.py $O/run_kernel_trace.csv 12 > $O/timeline.txt
