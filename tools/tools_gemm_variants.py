"""Where the x6 GEMM's time goes: structural variants (mrg_gemm_x6_variant) on the step's shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import _lib, functional as Fn  # noqa: E402

NAMES = {0: "x6 product", 1: "split + 1 MFMA", 2: "plane0 + 6 MFMA", 3: "plane0 + 1 MFMA (bf16 GEMM)"}


def main():
    lib = _lib.load()
    for (M, N, K) in [(19200, 1024, 256), (19200, 256, 256), (19200, 256, 1024), (4096, 4096, 4096)]:
        A = torch.randn(M, K, device="cuda")
        B = torch.randn(N, K, device="cuda")
        C = torch.zeros(M, N, device="cuda")
        for var in range(4):
            def go():
                _lib.check(lib.mrg_gemm_x6_variant(var, M, N, K, Fn._ptr(A), Fn._ptr(B), Fn._ptr(C), Fn._stream()), "v")
            for _ in range(3):
                go()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = 20
            e0.record()
            for _ in range(it):
                go()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / it * 1e3
            print(f"M={M:6d} N={N:5d} K={K:5d}  var {var} {NAMES[var]:30s} {us:8.1f} us  "
                  f"{2.0*M*N*K/us/1e6:7.1f} TF/s(fp32-eq)", flush=True)


if __name__ == "__main__":
    main()
