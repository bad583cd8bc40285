#!/bin/bash
# A/B of environment settings on one box: GPU tests (default env), then alternating bench runs.
#   ENVA="MRG_GEMM_GLDS=0 MRG_DX_TRANSPOSED=0" ENVB="" TESTS="tests/test_gpu_ops.py" bash tools/tools_gpu_envab.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/envab
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -m gpu -x -q -p no:cacheprovider --timeout 200 \
    --timeout-method thread > $R/gpurun_out/envab/tests.log 2>&1 || { tail -30 $R/gpurun_out/envab/tests.log; exit 1; }
  tail -1 $R/gpurun_out/envab/tests.log
fi
for i in 1 2; do
  for v in A B; do
    eval "E=\$ENV$v"
    env $E timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 --secondary ${SECONDARY:-0} $EXTRA \
      > $R/gpurun_out/envab/bench_${v}_$i.log 2>&1 || { tail -20 $R/gpurun_out/envab/bench_${v}_$i.log; exit 1; }
    python - $R/gpurun_out/envab/bench_${v}_$i.log "$v [$E]" $i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
line = f"{sys.argv[2]} run {sys.argv[3]} ms/step {d['ms_per_step']} " + " ".join(f"{n}={v['ms_per_step']}" for n, v in k.items())
for name, sec in d.get("secondary", {}).items():
    line += f" | {name} {sec['ms_per_step']}"
print(line)
PY
  done
done
