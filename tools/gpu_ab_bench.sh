#!/bin/bash
# A/B of the headline step on one box: alternating runs of bench.py (no secondary, no CPU baseline) under
# two or more environment settings ("-" = none).  bash tools/gpu_ab_bench.sh OUT REPS "ENV_A" "ENV_B" ...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
REPS=$2
shift 2
mkdir -p $O
for i in $(seq $REPS); do
  for e in "$@"; do
    ee=$e; [ "$e" = "-" ] && ee=""
    env $ee timeout -k 10 300 python $R/bench.py --secondary 0 --cpu-baseline 0 --steps 30 --warmup 5 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
    echo "$e: $(grep -o '"ms_per_step": [0-9.]*' $O/ab.json | head -1)"
  done
done
