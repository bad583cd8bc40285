#!/bin/bash
# A/B of schedule knobs on the headline bench (one box): stack chunk length, weight-gradient split target.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_ab
mkdir -p $O
cd $R
run() {
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --secondary 0 > $O/b.log 2>&1 \
    || { tail -5 $O/b.log; exit 1; }
  echo "$* $(grep -o '"ms_per_step": [0-9.]*' $O/b.log | head -1)"
}
for rep in 1 2; do
  run MRG_STACK_CHUNK=60
  run MRG_STACK_CHUNK=40
  run MRG_STACK_CHUNK=50
  run MRG_STACK_CHUNK=75
  run MRG_WGRAD_TARGET_WG=256
  run MRG_WGRAD_TARGET_WG=128
done
