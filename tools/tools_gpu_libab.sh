#!/bin/bash
# A/B of two library builds on one box: GPU tests on B, then alternating bench runs (A, B, A, B).
#   A=libmrg_old.so B=libmrg.so TESTS="tests/test_gpu_ops.py -k attention" bash tools/tools_gpu_libab.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P=$R/multimodalreactiongeneration_amd
mkdir -p $R/gpurun_out/libab
if [ -n "$TESTS" ]; then
  MRG_LIB_PATH=$P/$B timeout -k 10 400 python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -m gpu -x -q -p no:cacheprovider --timeout 200 \
    --timeout-method thread > $R/gpurun_out/libab/tests.log 2>&1 || { tail -30 $R/gpurun_out/libab/tests.log; exit 1; }
  tail -1 $R/gpurun_out/libab/tests.log
fi
for i in 1 2; do
  for L in $A $B; do
    MRG_LIB_PATH=$P/$L timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 --secondary 0 $EXTRA \
      > $R/gpurun_out/libab/bench_${L}_$i.log 2>&1 || { tail -20 $R/gpurun_out/libab/bench_${L}_$i.log; exit 1; }
    python - $R/gpurun_out/libab/bench_${L}_$i.log $L $i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], "run", sys.argv[3], "ms/step", d["ms_per_step"], " ".join(f"{n}={v['ms_per_step']}" for n, v in k.items()))
PY
  done
done
