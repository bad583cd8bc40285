#!/bin/bash
# round 4: bisect variants of the r03 replay failure; block-stack traces and A/B (chunk wgrads off)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_e
mkdir -p $O
cd $R
for v in b c; do
  timeout -k 10 300 python -u _bisect/diag_replay.py _bisect/$v > $O/bisect_$v.log 2>&1; echo "bisect $v rc=$?"
  grep -v amdgpu $O/bisect_$v.log | cut -c1-200
done
for i in 1 2; do
  for v in 0 1; do
    MRG_BLOCK_STACK=$v timeout -k 10 300 python -u bench.py --secondary 0 --cpu-baseline 0 --steps 30 > $O/bench_bs$v.$i.log 2>&1 || exit $?
    echo "block_stack=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_bs$v.$i.log | head -1)"
  done
done
for c in 75 150; do
  MRG_BLOCK_CHUNK=$c timeout -k 10 300 python -u bench.py --secondary 0 --cpu-baseline 0 --steps 30 > $O/bench_chunk$c.log 2>&1 || exit $?
  echo "block_chunk=$c: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_chunk$c.log | head -1)"
done
cd /tmp
for v in 0 1; do
  MRG_BLOCK_STACK=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bs$v -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/trace_bs$v.log 2>&1 \
    || { echo "trace $v failed"; tail -20 $O/trace_bs$v.log; exit 1; }
  echo "trace $v ok"
done
cd $R
for v in 0 1; do
  T=$(ls $O/trace_bs$v/*/run_kernel_trace.csv $O/trace_bs$v/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/tools_timeline.py $T 2 > $O/timeline_bs$v.txt
  head -25 $O/timeline_bs$v.txt
done
