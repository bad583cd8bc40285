#!/bin/bash
# A/B of one bench flag on one box: tests first, then alternating bench runs, then a kernel trace of B.
#   FLAG=--wgrad-defer A=0 B=1 TESTS="tests/test_gpu_models.py -k side_stream" bash tools/tools_gpu_ab2.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ab
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    > $R/gpurun_out/ab/tests.log 2>&1 || { tail -30 $R/gpurun_out/ab/tests.log; exit 1; }
  tail -1 $R/gpurun_out/ab/tests.log
fi
for i in 1 2; do
  for v in $A $B; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 --secondary 0 $FLAG $v $EXTRA \
      > $R/gpurun_out/ab/bench_${v}_$i.log 2>&1 || { tail -20 $R/gpurun_out/ab/bench_${v}_$i.log; exit 1; }
    echo "$FLAG $v run $i: $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/ab/bench_${v}_$i.log)"
  done
done
if [ "${TRACE:-1}" = "1" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab/trace -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 $FLAG $B $EXTRA > $R/gpurun_out/ab/trace.log 2>&1 \
    || { echo "trace failed"; tail -5 $R/gpurun_out/ab/trace.log; exit 1; }
  echo "trace ok"
fi
