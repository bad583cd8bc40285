#!/bin/bash
# round 4: block stack now eligible: parity tests, A/B over chunk sizes; capture diag (deferral off)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_models.py tests/test_gpu_capture.py -k "block_stack or b64 or replayed_step or kv_sink" -s > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|worst|Error|assert" $O/tests.log | head -20; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    MRG_BLOCK_STACK=$v timeout -k 10 300 python -u bench.py --secondary 0 --cpu-baseline 0 --steps 30 > $O/bench_bs$v.$i.log 2>&1 || exit $?
    echo "block_stack=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_bs$v.$i.log | head -1)"
  done
done
for c in 60 75 150; do
  MRG_BLOCK_CHUNK=$c timeout -k 10 300 python -u bench.py --secondary 0 --cpu-baseline 0 --steps 30 > $O/bench_chunk$c.log 2>&1 || exit $?
  echo "block_chunk=$c: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_chunk$c.log | head -1)"
done
timeout -k 10 600 python -u tools/tools_capture_diag.py > $O/capture_diag.log 2>&1; echo "diag rc=$?"; grep -v amdgpu $O/capture_diag.log | cut -c1-250
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bs1 -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/trace_bs1.log 2>&1 \
    || { echo "trace failed"; tail -20 $O/trace_bs1.log; exit 1; }
cd $R
T=$(ls $O/trace_bs1/*/run_kernel_trace.csv $O/trace_bs1/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/tools_timeline.py $T 2 > $O/timeline_bs1.txt
head -22 $O/timeline_bs1.txt
