#!/bin/bash
# GPU round-trip used during development: tests, bench, kernel profile (each step bounded).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
echo "tests exit $?" >> gpurun_out/gpu_tests.log
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --graph 0 --cpu-baseline 0 --steps 3 --warmup 1 > $R/gpurun_out/prof.log 2>&1
  echo "prof exit $?"
fi
