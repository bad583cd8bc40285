"""Per-product time of the LDS-DMA x6 kernels vs the warp-specialized ones (gemm_wsp.hip) on the
step's shapes: weight gradients dW = dY^T X and k-contiguous products C = A W^T.

    python tools/tools_wsp_bench.py          (GPU box)
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import _lib as L  # noqa: E402
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    lib = L.load()
    dev = torch.device("cuda:0")
    VP = ctypes.c_void_p
    Fn.set_wgrad_stream(False)
    print("weight gradients (rows x Nout x Nin): us per product, LDS-DMA vs specialized", flush=True)
    for rows, N, In in ((19200, 1024, 256), (19200, 256, 256), (19200, 512, 256), (19200, 256, 512),
                        (6400, 1024, 256)):
        dy, x = torch.randn(rows, N, device=dev), torch.randn(rows, In, device=dev)
        gw, gb = torch.zeros(N, In, device=dev), torch.zeros(N, device=dev)
        res = []
        for wsp in (0, 1):
            old = lib.mrg_gemm_set_wgrad_kernel(wsp)
            res.append(timeit(lambda: Fn._wgrad(Fn._ptr(dy), N, Fn._ptr(x), In, rows, N, In, gw, dev, gb=gb,
                                                keep=(dy, x))))
            lib.mrg_gemm_set_wgrad_kernel(old)
        fl = 2.0 * rows * N * In
        print(f"  {rows} x {N} x {In}: {res[0]:8.1f} us ({fl / res[0] / 1e6:6.1f} TF/s)  "
              f"{res[1]:8.1f} us ({fl / res[1] / 1e6:6.1f} TF/s)", flush=True)
    print("k-contiguous products (M x N x K): us per product, LDS-DMA vs specialized", flush=True)
    for M, N, K in ((19200, 1024, 256), (19200, 256, 256), (19200, 512, 256), (19200, 256, 1024),
                    (19200, 256, 512), (6400, 1024, 256)):
        A, W = torch.randn(M, K, device=dev), torch.randn(N, K, device=dev) / 16
        b, C = torch.randn(N, device=dev), torch.empty(M, N, device=dev)
        res = []
        for wsp in (0, 2):
            old = lib.mrg_gemm_set_wgrad_kernel(wsp)
            res.append(timeit(lambda: L.check(lib.mrg_gemm_f32_ex(
                M, N, K, 1.0, VP(A.data_ptr()), 0, K, 0, 0, VP(W.data_ptr()), 1, K, 0, 0, 0.0, VP(C.data_ptr()), N,
                VP(b.data_ptr()), 0, None, N, None, 1, None, None, 0.0, None, Fn._stream()), "gemm")))
            lib.mrg_gemm_set_wgrad_kernel(old)
        fl = 2.0 * M * N * K
        print(f"  {M} x {N} x {K}: {res[0]:8.1f} us ({fl / res[0] / 1e6:6.1f} TF/s)  "
              f"{res[1]:8.1f} us ({fl / res[1] / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
