#!/bin/bash
# Kernel times + SQ counters of the attention kernels (tools_attn_bench.py), one pass per counter set.
#   VARIANTS="0 1" bash tools/tools_gpu_attn_sq.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/asq
mkdir -p $O
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- \
  python3 $R/tools/tools_attn_bench.py $VARIANTS > $O/kt.log 2>&1 || { echo "trace failed"; tail -5 $O/kt.log; exit 1; }
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o p --output-format csv -- python3 $R/tools/tools_attn_bench.py $VARIANTS \
    > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for f in glob.glob(o + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "attn" in r["Name"]:
            print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:8.1f}")
vals = collections.defaultdict(list)
for f in glob.glob(o + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "attn" in r["Kernel_Name"]:
            vals[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    print(f"{k:60s} {c:28s} {sum(v)/len(v):14.0f}")
PY
