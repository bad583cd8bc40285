#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gemm_ns
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/tools_gemm_ns.py > $O/ns.log 2>&1 || { tail -20 $O/ns.log; exit 1; }
cat $O/ns.log
