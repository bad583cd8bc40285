#!/bin/bash
# round 4: block wavefront parity + A/B
set -o pipefail
O=gpurun_out/r04_c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ops.py tests/test_gpu_models.py -k "query_chunks or block_stack or b64 or timeout_reports" -s > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    MRG_BLOCK_STACK=$v timeout -k 10 300 python -u bench.py --secondary 0 --cpu-baseline 0 --steps 30 > $O/bench_bs$v.$i.log 2>&1 || exit $?
    echo "block_stack=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_bs$v.$i.log | head -1)"
  done
done
