#!/bin/bash
# Alternating A/B bench runs (no tests, no CPU baseline): A = defaults, B = ${AB_ARGS}; 3 rounds.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then X=""; else X="${AB_ARGS}"; fi
    timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline 0 $X > gpurun_out/bench_$v$i.log 2>&1 || { tail -20 gpurun_out/bench_$v$i.log; exit 1; }
    python -c "import json,sys;d=json.loads(open('gpurun_out/bench_$v$i.log').read().strip().splitlines()[-1]);print('$v$i', d['ms_per_step'])"
  done
done
