"""Run one GEMM shape repeatedly (for rocprofv3 counter passes): python tools_gemm_one.py M N K ta tb [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from tools_gemm_bench import run_shape  # noqa: E402

M, N, K, ta, tb = (int(x) for x in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 10
ms, splits, err = run_shape(M, N, K, ta, tb, False, iters=iters)
print(f"M={M} N={N} K={K} ta={ta} tb={tb}: {ms*1e3:.1f} us  {2.0*M*N*K/(ms/1e3)/1e12:.1f} TF/s")
