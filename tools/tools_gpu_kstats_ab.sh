#!/bin/bash
# Per-kernel average durations of the default bench workload under two library builds (kernel trace).
#   A=libmrg_old.so B=libmrg.so KPAT="resln_param|attn" bash tools/tools_gpu_kstats_ab.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P=$R/multimodalreactiongeneration_amd
O=$R/gpurun_out/kab
mkdir -p $O
cd /tmp
for L in $A $B; do
  MRG_LIB_PATH=$P/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$L -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --secondary 0 > $O/$L.log 2>&1 \
    || { echo "trace $L failed"; tail -20 $O/$L.log; exit 1; }
  python3 - $O/$L "$KPAT" $L <<'PY'
import csv, glob, re, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if re.search(sys.argv[2], r["Name"]):
            print(f"{sys.argv[3]:16s} {r['Name'][:70]:70s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:8.2f}")
PY
done
