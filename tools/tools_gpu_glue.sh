#!/bin/bash
# GPU tests + one short kernel trace of the headline bench: lists the non-library (at::native)
# kernels left in the replayed step.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/glue
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
cd $R
S=$(ls $O/trace/*/run_kernel_stats.csv $O/trace/run_kernel_stats.csv 2>/dev/null | head -1)
python3 - $S <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "mrg::" not in n:
        print(r["Calls"], n[:110])
PY
