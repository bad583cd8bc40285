#!/bin/bash
# A/B of environment settings on the headline bench: bash tools/tools_gpu_envab.sh "" "MRG_X=1" ...
# (each setting twice, interleaved; "" = defaults)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/envab
mkdir -p $O
cd $R
for rep in 1 2; do
  for setting in "$@"; do
    env $setting timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --secondary 0 > $O/b.log 2>&1 \
      || { tail -5 $O/b.log; exit 1; }
    echo "[$setting] $(grep -o '"ms_per_step": [0-9.]*' $O/b.log | head -1)"
  done
done
