mkdir -p gpurun_out/r05_p3 && O=gpurun_out/r05_p3 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "attention or param_reduce" > $O/attn_t.log 2>&1; tail -3 $O/attn_t.log; \
grep -q " passed" $O/attn_t.log && ! grep -q "failed\|error" $O/attn_t.log && \
timeout -k 10 120 env MRG_ATTN_FUSED=1 python -u tools/tools_attn_bench.py 3 > $O/attn_b1.log 2>&1 && \
timeout -k 10 120 env MRG_ATTN_FUSED=0 python -u tools/tools_attn_bench.py 3 > $O/attn_b0.log 2>&1 ; \
grep -v amdgpu $O/attn_b1.log | tail -4; grep -v amdgpu $O/attn_b0.log | tail -4; \
timeout -k 10 200 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_models.py -k "persistent_forward" > $O/persist_t.log 2>&1 ; tail -2 $O/persist_t.log; \
timeout -k 10 120 env MRG_SSD_PERSIST=1 python -u tools/ssd_stamps.py > $O/persist_s.log 2>&1; grep -v amdgpu $O/persist_s.log | tail -25; \
bash tools/gpu_ab_bench.sh r05_p3 2 - MRG_ATTN_FUSED=0 MRG_TAIL_SIDE=2 MRG_TAIL_SIDE=4
