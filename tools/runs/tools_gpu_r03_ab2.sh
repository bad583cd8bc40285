#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_ab2
mkdir -p $O
cd $R
run() {
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --secondary 0 "$@" > $O/b.log 2>&1 \
    || { tail -5 $O/b.log; exit 1; }
  echo "$* $(grep -o '"ms_per_step": [0-9.]*' $O/b.log | head -1)"
}
for rep in 1 2; do
  run --wgrad-defer 0
  run --wgrad-defer 1
done
