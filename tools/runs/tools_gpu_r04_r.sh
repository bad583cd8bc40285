#!/bin/bash
# round 4: kernel census of C2 simple_lstm fp32 and bf16 (graph-replayed steps)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_r
mkdir -p $O
cd /tmp
for p in 32 bf16; do
  C2_PRECISION=$p timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/c2_$p -o run -- \
    python3 $R/tools/tools_bench_models.py 5 C2 1 > $O/c2_$p.log 2>&1 || { echo "trace $p failed"; tail -5 $O/c2_$p.log; exit 1; }
  cp /tmp/c2_$p/run_kernel_stats.csv $O/c2_${p}_stats.csv
  grep -o '{"C2.*' $O/c2_$p.log | tail -1
done
