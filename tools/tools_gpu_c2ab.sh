#!/bin/bash
# C2 (simple_lstm fp32 / bf16) step times per environment setting: bash tools/tools_gpu_c2ab.sh "" "MRG_X=1"
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c2ab
cd $R
for setting in "$@"; do
  env $setting timeout -k 10 200 python -u tools/tools_c2_prof.py > gpurun_out/c2ab/log.txt 2>&1 || { tail -5 gpurun_out/c2ab/log.txt; exit 1; }
  echo "[$setting] $(grep C2 gpurun_out/c2ab/log.txt | tr '\n' ' ')"
done
