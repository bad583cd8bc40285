#!/bin/bash
# round 4: block stack with per-chunk dQ + one dK/dV pass per block; backward MX threshold A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_g
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ops.py tests/test_gpu_models.py -k "query_chunks or block_stack or b64" -s > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|worst|Error|assert" $O/tests.log | head -20; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --secondary 0 --cpu-baseline 0 --steps 30 > $O/bench_$n.log 2>&1 || exit $?
  echo "$n: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$n.log | head -1)"
}
for i in 1 2; do
  run bs0.$i MRG_BLOCK_STACK=0
  run bs1.$i MRG_BLOCK_STACK=1
  run bs1_bwd8.$i MRG_BLOCK_STACK=1 MRG_LSTM_MX_MIN_BS_BWD=8
done
run bs1_c150 MRG_BLOCK_STACK=1 MRG_BLOCK_CHUNK=150
run bs1_c150_bwd8 MRG_BLOCK_STACK=1 MRG_BLOCK_CHUNK=150 MRG_LSTM_MX_MIN_BS_BWD=8
run bs1_c75_bwd8 MRG_BLOCK_STACK=1 MRG_BLOCK_CHUNK=75 MRG_LSTM_MX_MIN_BS_BWD=8
run bs0_bwd8 MRG_BLOCK_STACK=0 MRG_LSTM_MX_MIN_BS_BWD=8
cd /tmp
export MRG_BLOCK_STACK=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bs1 -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/trace_bs1.log 2>&1 \
    || { echo "trace failed"; tail -20 $O/trace_bs1.log; exit 1; }
export MRG_BLOCK_STACK=0
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bs0 -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/trace_bs0.log 2>&1 \
    || { echo "trace failed"; tail -20 $O/trace_bs0.log; exit 1; }
cd $R
for v in bs1 bs0; do
  T=$(ls $O/trace_$v/*/run_kernel_trace.csv $O/trace_$v/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/tools_timeline.py $T 2 > $O/timeline_$v.txt
  echo "== $v"; head -19 $O/timeline_$v.txt
done
