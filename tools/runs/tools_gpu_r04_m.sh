#!/bin/bash
# round 4: paired SimpleLSTM encoders (one recurrence launch per block for both encoders)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_m
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_ops.py \
  -k "simple or lstm_solo or bidirectional or batched_problems" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|assert" $O/tests.log | tail -6; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  MRG_PAIR_ENCODERS=$v timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --cpu-baseline 0 > $O/bench_pair$v.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_pair$v.log; exit 1; }
  echo "pair=$v: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_pair$v.log | head -1)"
  python3 - $O/bench_pair$v.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
for k, v in (d.get("secondary") or {}).items():
    if isinstance(v, dict): print(f"  {k}: {v.get('ms_per_step')} ms/step")
PY
done
