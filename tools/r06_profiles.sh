#!/bin/bash
# Round-6 profile set (gpurun -- bash tools/r06_profiles.sh <tag>): GPU tests + smoke, the
# default bench line (secondary configs, CPU baselines), a kernel trace of the bench's headline
# workload (graph replayed) -> trace roofline summary, FETCH_SIZE / WRITE_SIZE passes over one eager
# step -> PMC summary.  Every GPU step has its own limit; the script stops at the first failure.
# PART=1: GPU tests + smoke; PART=2: bench, trace, PMC, stamps; PART=3: kernel census of the C3 step
# and of generation (tools/c3_census.py under rocprofv3); PART=4: the final set (tests, smoke, trace
# installed as the committed trace summary, then the bench line that checks against it).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-v1}
O=$R/gpurun_out/r06_$TAG
mkdir -p $O
cd $R
if [ "${PART:-1}" = "4" ]; then
# final set: GPU tests + smoke, then the kernel trace FIRST, its summary installed as the committed
# profiles/r06_trace_roofline.json that the bench line's trace_check reads, then the default bench line
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/trace.log 2>&1 \
  || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
cd $R
T=$(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/tools_trace_roofline.py $T $O/trace_roofline.json > /dev/null
cp $O/trace_roofline.json profiles/r06_trace_roofline.json
python3 tools/tools_timeline.py $T 2 > $O/timeline.txt
S=$(ls $O/trace/*/run_kernel_stats.csv $O/trace/run_kernel_stats.csv 2>/dev/null | head -1)
python3 tools/tools_prof_summary.py $S > $O/kernel_summary.txt 2>/dev/null || cp $S $O/kernel_stats.csv
echo "trace ok"
timeout -k 10 600 python bench.py > $O/bench.json.log 2>&1 || { tail -20 $O/bench.json.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench.json.log | tail -1
exit 0
fi
if [ "${PART:-1}" = "3" ]; then
cd /tmp
for w in c3 gen; do
  reps=$([ $w = c3 ] && echo 10 || echo 3)
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/census_$w -o run -- \
    python3 $R/tools/c3_census.py $w $reps > $O/census_$w.log 2>&1 || { echo "census $w failed"; tail -20 $O/census_$w.log; exit 1; }
  S=$(ls $O/census_$w/*/run_kernel_stats.csv $O/census_$w/run_kernel_stats.csv 2>/dev/null | head -1)
  python3 $R/tools/tools_prof_summary.py $S $((reps + 2)) 30 > $O/census_$w.txt
  grep ms/step $O/census_$w.log; tail -1 $O/census_$w.txt
done
exit 0
fi
if [ "${PART:-1}" = "1" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
exit 0
fi
timeout -k 10 600 python bench.py > $O/bench.json.log 2>&1 || { tail -20 $O/bench.json.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench.json.log | head -1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/trace.log 2>&1 \
  || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
echo "trace ok"
for c in $([ "${PMC:-1}" = "1" ] && echo FETCH_SIZE WRITE_SIZE); do
  timeout -k 10 400 rocprofv3 --pmc $c -d $O/pmc/$c -o pmc --output-format csv -- \
    python3 $R/bench.py --graph 0 --wgrad-stream 0 --cpu-baseline 0 --secondary 0 --steps 1 --warmup 1 \
    > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -20 $O/pmc_$c.log; exit 1; }
  echo "pmc $c ok"
done
cd $R
T=$(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/tools_trace_roofline.py $T $O/trace_roofline.json > /dev/null
python3 tools/tools_timeline.py $T 2 > $O/timeline.txt
S=$(ls $O/trace/*/run_kernel_stats.csv $O/trace/run_kernel_stats.csv 2>/dev/null | head -1)
python3 tools/tools_prof_summary.py $S > $O/kernel_summary.txt 2>/dev/null || cp $S $O/kernel_stats.csv
cat $O/timeline.txt | head -30
[ "${STAMPS:-1}" = "1" ] || exit 0
timeout -k 10 200 env MX=2 STAMP_CFGS=1:0,3:0,8:0 python -u tools/tools_lstm_stamps.py > $O/mx_stamps.log 2>&1 || { tail -5 $O/mx_stamps.log; exit 1; }
timeout -k 10 200 env STAMP_CFGS=1:0,2:0 python -u tools/tools_lstm_stamps.py > $O/valu_stamps.log 2>&1 || { tail -5 $O/valu_stamps.log; exit 1; }
grep -E "fwd|bwd" $O/mx_stamps.log $O/valu_stamps.log
