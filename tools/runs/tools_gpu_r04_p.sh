#!/bin/bash
# round 4: one-barrier solo forward recurrence: LSTM op tests, per-step A/B, C2 bench
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_p
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py \
  -k "lstm or simple" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  MRG_LSTM_SOLO1=$v timeout -k 10 300 python -u tools/tools_lstm_solo.py > $O/solo1_$v.log 2>&1 || { tail -5 $O/solo1_$v.log; exit 1; }
  echo "== solo1=$v"; grep -v amdgpu $O/solo1_$v.log
done
H=128 STAMP_CFGS=1:0 timeout -k 10 300 python -u tools/tools_lstm_stamps.py > $O/stamps128.log 2>&1 || exit 1
grep -E "^fwd|^bwd" $O/stamps128.log
for v in 0 1; do
  MRG_LSTM_SOLO1=$v timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --cpu-baseline 0 > $O/bench_solo1_$v.log 2>&1 || { tail -5 $O/bench_solo1_$v.log; exit 1; }
  echo "solo1=$v: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_solo1_$v.log | head -1)"
  python3 - $O/bench_solo1_$v.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
for k, v in (d.get("secondary") or {}).items():
    if isinstance(v, dict): print(f"  {k}: {v.get('ms_per_step')} ms/step")
PY
done
