mkdir -p gpurun_out/r05_p4 && O=gpurun_out/r05_p4 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "attention" > $O/attn_t.log 2>&1; tail -3 $O/attn_t.log; \
grep -q " passed" $O/attn_t.log && ! grep -q "failed\|error" $O/attn_t.log && \
timeout -k 10 120 env MRG_ATTN_FUSED=1 python -u tools/tools_attn_bench.py 3 > $O/attn_b1.log 2>&1 && \
grep -v amdgpu $O/attn_b1.log | tail -3 && \
bash tools/gpu_ab_bench.sh r05_p4 2 - MRG_ATTN_FUSED=0
