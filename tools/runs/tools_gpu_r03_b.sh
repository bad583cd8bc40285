#!/bin/bash
# Round-3 batched encoder-stack check: new op tests + stack tests, benches of both schedules, a
# kernel trace of the stack step.  Each GPU step has its own limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03b
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "batched or occupying or encoder_stack or mfma" > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for v in base stack; do
  E=""; [ $v = stack ] && E="MRG_ENCODER_STACK=1"
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --secondary 0 > $O/bench_$v.log 2>&1 \
    || { tail -20 $O/bench_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log | head -1
done
cd /tmp
MRG_ENCODER_STACK=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stack -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/stack_prof.log 2>&1 \
  || { echo "stack prof failed"; tail -5 $O/stack_prof.log; exit 1; }
cd $R
python3 tools/tools_timeline.py $(ls $O/stack/*/run_kernel_trace.csv $O/stack/run_kernel_trace.csv 2>/dev/null | head -1) 1 > $O/stack.timeline.txt
cat $O/stack.timeline.txt
