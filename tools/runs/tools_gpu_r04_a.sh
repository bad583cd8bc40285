#!/bin/bash
# round 4, first GPU call: new parity tests, capture diagnostics, launch-gap probe, --gpus check, headline
set -o pipefail
O=gpurun_out/r04_a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_capture.py \
  "tests/test_gpu_models.py::test_benchmark_schedule_b64_vs_oracle" \
  "tests/test_gpu_models.py::test_encoder_stack_mfma_matches_per_layer_valu" \
  "tests/test_gpu_models.py::test_simple_lstm_configs0_shape_vs_oracle" -s > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/tools_launch_gap.py > $O/launch_gap.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/tools_capture_diag.py > $O/capture_diag.log 2>&1 || exit $?
timeout -k 10 120 python -u bench.py --gpus 2 > $O/gpus2.log 2>&1; echo "bench --gpus 2 rc=$? (want 2)"
timeout -k 10 600 python -u bench.py --secondary 0 --cpu-baseline 0 > $O/bench.json.log 2>&1 || exit $?
tail -c 600 $O/bench.json.log
