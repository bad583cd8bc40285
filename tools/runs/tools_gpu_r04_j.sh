#!/bin/bash
# round 4: solo LSTM groups at H <= 128: op parity tests, per-step cost, C2 / C3 secondary bench
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_j
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py \
  -k "lstm" > $O/tests_ops.log 2>&1
rc=$?; echo "op tests rc=$rc"; grep -E "passed|failed|Error" $O/tests_ops.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/tools_lstm_solo.py > $O/solo.log 2>&1 || { echo "solo tool failed"; tail -20 $O/solo.log; exit 1; }
grep -v amdgpu $O/solo.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_models.py \
  -k "simple or sampling or golden or c3 or generation" > $O/tests_models.log 2>&1
rc=$?; echo "model tests rc=$rc"; grep -E "passed|failed|Error" $O/tests_models.log | tail -5; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  MRG_LSTM_SOLO=$v timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --cpu-baseline 0 > $O/bench_solo$v.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_solo$v.log; exit 1; }
  echo "solo=$v: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_solo$v.log | head -1)"
  python3 - $O/bench_solo$v.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
for k, v in (d.get("secondary") or {}).items():
    print(f"  {k}: {v.get('ms_per_step')} ms/step" if isinstance(v, dict) else f"  {k}: {v}")
PY
done
