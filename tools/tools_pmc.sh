#!/bin/bash
# HBM traffic per kernel from rocprofv3 PMC counters: one pass per counter (FETCH_SIZE and
# WRITE_SIZE do not fit one TCC pass on gfx950), kernel dispatch data only, eager steps.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c -d $R/gpurun_out/pmc/$c -o pmc --output-format csv -- python3 $R/bench.py --graph 0 --wgrad-stream 0 --cpu-baseline 0 --steps 1 --warmup 1 > $R/gpurun_out/pmc/$c.log 2>&1 || { echo "pmc $c failed"; tail -20 $R/gpurun_out/pmc/$c.log; exit 1; }
  echo "pmc $c ok"
done
