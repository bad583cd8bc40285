# rocprof kernel traces of the default step and the encoder-stack step (graph-replayed)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03/prof
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/base.log 2>&1 || { echo "base failed"; tail -5 $O/base.log; exit 1; }
echo base ok
MRG_ENCODER_STACK=1 MRG_STACK_MAXP=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stack -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/stack.log 2>&1 || { echo "stack failed"; tail -5 $O/stack.log; exit 1; }
echo stack ok
cd $R
for v in base stack; do f=$(ls $O/$v/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls $O/$v/run_kernel_trace.csv); python3 tools/tools_timeline.py $f 2 > $O/$v.timeline.txt; done
