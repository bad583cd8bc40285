#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_ab3
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "weight_grad or side_stream or layernorm or handoff or adamw" > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --secondary 0 "$@" > $O/b.log 2>&1 \
    || { tail -5 $O/b.log; exit 1; }
  echo "$* $(grep -o '"ms_per_step": [0-9.]*' $O/b.log | head -1)"
}
for rep in 1 2; do
  run --wgrad-defer 0
  run --wgrad-defer 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
cd $R
python3 tools/tools_timeline.py $(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1) 1
