#!/bin/bash
# SQ counters over one eager training step (bench.py --graph 0), two passes; per-kernel summary by
# tools_sq_summary.py.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/spmc
cd /tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d $R/gpurun_out/spmc/p$i -o p --output-format csv -- python3 $R/bench.py --graph 0 --cpu-baseline 0 --steps 1 --warmup 1 > $R/gpurun_out/spmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/spmc/p$i.log; exit 1; }
  echo "pass $i ok"
done
