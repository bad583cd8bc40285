#!/bin/bash
# round 4: what the VALU forward's Gx prefetch wait costs — stamps with the prefetch vs re-reading the
# current step's Gx (MRG_DBG_GX_PIN=1, timing only)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_ae
mkdir -p $O
cd $R
for v in 0 1 0 1; do
  MRG_DBG_GX_PIN=$v STAMP_CFGS=1:0,2:0 timeout -k 10 200 python -u tools/tools_lstm_stamps.py > $O/stamps_$v.log 2>&1 || { tail -5 $O/stamps_$v.log; exit 1; }
  echo "pin=$v"; grep -E "^fwd|launch" $O/stamps_$v.log
done
