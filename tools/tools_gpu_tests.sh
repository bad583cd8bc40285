#!/bin/bash
# the GPU test suite (own time limit), then the default bench twice
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tests
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/tools_gpu_envab.sh ""
