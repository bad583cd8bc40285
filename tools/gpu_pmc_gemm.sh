#!/bin/bash
# PMC passes over one planes GEMM shape per kernel config: bash tools/gpu_pmc_gemm.sh OUT M N K cfg...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1; shift
M=$1; N=$2; K=$3; shift 3
mkdir -p $O
cd /tmp
for cfg in "$@"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_$cfg -o run --output-format csv -- python3 $R/tools/gemm_one.py $M $N $K $cfg 20 > $O/kt_$cfg.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS -d $O/pmc1_$cfg -o pmc --output-format csv -- python3 $R/tools/gemm_one.py $M $N $K $cfg 5 > $O/pmc1_$cfg.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/pmc2_$cfg -o pmc --output-format csv -- python3 $R/tools/gemm_one.py $M $N $K $cfg 5 > $O/pmc2_$cfg.log 2>&1 || exit 1
done
echo done
