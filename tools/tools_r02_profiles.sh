#!/bin/bash
# Round-2 profile set (run on a GPU box: gpurun -- bash tools/tools_r02_profiles.sh):
#   1. kernel trace + stats of the default bench command's workload (graph replayed, one stream
#      for the probe steps), 2. FETCH_SIZE / WRITE_SIZE passes over one eager step (tools_pmc.sh),
#   3. the access-pattern calibration of those counters (tools/pmc_calib).
# Every GPU step runs under its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02
mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/trace.log 2>&1 \
  || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
echo "trace ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c -d $O/pmc/$c -o pmc --output-format csv -- \
    python3 $R/bench.py --graph 0 --wgrad-stream 0 --cpu-baseline 0 --secondary 0 --steps 1 --warmup 1 \
    > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -20 $O/pmc_$c.log; exit 1; }
  echo "pmc $c ok"
done
for c in $([ -x $R/tools/pmc_calib ] && echo FETCH_SIZE WRITE_SIZE); do
  timeout -k 10 120 rocprofv3 --pmc $c -d $O/calib/$c -o pmc --output-format csv -- $R/tools/pmc_calib \
    > $O/calib_$c.log 2>&1 || { echo "calib $c failed"; tail -20 $O/calib_$c.log; exit 1; }
  echo "calib $c ok"
done
