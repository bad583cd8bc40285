"""fp32 GEMM throughput of the vendor library (torch.matmul -> hipBLASLt / rocBLAS) vs the x6 kernels on
the step's product shapes: is a library fp32 GEMM a better base than the three-plane bf16 split?

    python tools/tools_blas_fp32.py          (GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3   # us


def main():
    dev = "cuda:0"
    torch.backends.cuda.matmul.allow_tf32 = False
    for M, N, K, what in ((19200, 1024, 256, "LSTM Gx  x W_ih^T"), (19200, 256, 256, "E x E"),
                          (19200, 256, 1024, "dG W_ih"), (1024, 256, 19200, "dW_ih = dG^T x"),
                          (256, 256, 19200, "dW (E x E)")):
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev)
        c = torch.empty(M, N, device=dev)
        t_lib = timeit(lambda: torch.matmul(a, w.t(), out=c))
        t_x6 = timeit(lambda: Fn.linear(a, w, None))
        ref = (a.double() @ w.double().t())
        e_lib = ((c.double() - ref).abs().max() / ref.abs().max()).item()
        e_x6 = ((Fn.linear(a, w, None).double() - ref).abs().max() / ref.abs().max()).item()
        fl = 2.0 * M * N * K
        print(f"{what:18s} {M}x{N}x{K}: library {t_lib:7.1f} us {fl / t_lib / 1e6:6.1f} TF/s err {e_lib:.1e} | "
              f"x6 {t_x6:7.1f} us {fl / t_x6 / 1e6:6.1f} TF/s err {e_x6:.1e}", flush=True)


if __name__ == "__main__":
    main()
