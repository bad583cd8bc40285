#!/bin/bash
# MX recurrence change check: parity tests touching the MFMA form, stamps, bench.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_mx
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "mfma or encoder_stack or occupying or fused_integrator or benchmark_width" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 env MX=2 STAMP_CFGS=1:0,8:0 python -u tools/tools_lstm_stamps.py > $O/mx_stamps.log 2>&1 || { tail -5 $O/mx_stamps.log; exit 1; }
grep -E "fwd|bwd" $O/mx_stamps.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --secondary 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench.log | head -1
