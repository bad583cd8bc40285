#!/bin/bash
# round 4: bisect the r03 replay failure on the pre-fix tree; tests of the sink / per-chunk wgrads; A/B
set -o pipefail
O=gpurun_out/r04_b
mkdir -p $O
timeout -k 10 300 python -u _bisect/diag_replay.py _bisect/a > $O/bisect_a.log 2>&1; echo "bisect rc=$?"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_capture.py tests/test_gpu_models.py tests/test_gpu_ops.py \
  -k "query_chunks or layernorm or encoder_stack or b64 or kv_sink or feature_input or fused_integrator or wgrad_side or benchmark_width" -s > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    MRG_STACK_CHUNK_WGRAD=$v timeout -k 10 300 python -u bench.py --secondary 0 --cpu-baseline 0 --steps 30 > $O/bench_cw$v.$i.log 2>&1 || exit $?
    echo "chunk_wgrad=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_cw$v.$i.log | head -1)"
  done
done
timeout -k 10 300 python -u tools/tools_lstm_multi.py > $O/lstm_multi.log 2>&1; echo "lstm_multi rc=$?"
