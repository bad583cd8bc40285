#!/bin/bash
# Round-3 state check: GPU tests, MX/stack parity diagnostic, benches of the default step and the
# encoder-stack step, kernel traces of both.  Every GPU step has its own time limit; stops at the
# first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u tools/tools_mx_parity.py > $O/mx_parity.log 2>&1 || { tail -20 $O/mx_parity.log; exit 1; }
cat $O/mx_parity.log
for v in base stack; do
  E=""; [ $v = stack ] && E="MRG_ENCODER_STACK=1"
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --secondary 0 > $O/bench_$v.log 2>&1 \
    || { tail -20 $O/bench_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log | head -1
done
bash tools/runs/tools_gpu_r03_prof.sh
