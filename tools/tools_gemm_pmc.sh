#!/bin/bash
# SQ counters for two GEMM shapes (short-K model shape vs long-K square), one pass per counter group.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/gpmc
cd /tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for shape in ${GPMC_SHAPES:-"19200 1024 256 0 1"}; do
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $P -d $R/gpurun_out/gpmc/p$i -o p --output-format csv -- python3 $R/tools/tools_gemm_one.py $shape 5 > $R/gpurun_out/gpmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/gpmc/p$i.log; exit 1; }
    echo "pass $i ($shape) ok"
  done
done
