"""LDS-DMA x6 GEMM (gemm_x6g_kernel) per ring depth / column tile on the step's k-contiguous shapes,
beside a copy of the same bytes (A read + C write) as the memory floor.

    python tools/tools_gemm_ns.py           (on a GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import functional as Fn, _lib  # noqa: E402

R = 64 * 300
SHAPES = [("lin256", R, 256, 256), ("kv512", R, 512, 256), ("gx1024", R, 1024, 256),
          ("cat512", R, 256, 512), ("dx1024", R, 256, 1024), ("ffn64", R, 64, 256)]


def timeit(fn, iters=30):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    lib = _lib.load()
    dev = "cuda:0"
    for name, M, N, K in SHAPES:
        A = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev)
        C = torch.empty(M, N, device=dev)
        src = torch.empty(M, K + N, device=dev)
        dst = torch.empty_like(src)
        cp = timeit(lambda: dst.copy_(src))
        ref = A.double() @ W.double().t()
        line = [f"{name:7s} {M}x{N}x{K}: copy(A+C bytes) {cp:6.1f} us"]
        for ns in (2, 3, 4):
            for bn in (128, 64):
                _lib.check(lib.mrg_gemm_set_glds(ns, bn), "glds")
                us = timeit(lambda: Fn.gemm(M, N, K, Fn._ptr(A), 0, K, Fn._ptr(W), 1, K, Fn._ptr(C), N, device=A.device))
                err = ((C.double() - ref).abs().max() / ref.abs().max()).item()
                tf = 2.0 * M * N * K / us / 1e6
                line.append(f"ns{ns}/bn{bn} {us:6.1f} us {tf:5.0f} TF err {err:.0e}")
        _lib.check(lib.mrg_gemm_set_glds(2, 128), "glds")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
