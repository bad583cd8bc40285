#!/bin/bash
# Round-trip: GPU tests, bench (with CPU baseline), kernel-trace profile, PMC traffic passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --graph 0 --wgrad-stream 0 --cpu-baseline 0 --steps 3 --warmup 1 > $R/gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -5 $R/gpurun_out/prof.log; exit 1; }
echo "prof ok"
cd $R
if [ "${PMC:-1}" = "1" ]; then bash tools/tools_pmc.sh; fi
