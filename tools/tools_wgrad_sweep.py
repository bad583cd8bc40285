"""Weight-gradient products dW = dY^T X (K = B*T = 19200 rows) per split-K factor, with the grid
uncapped and capped at one block per CU (how they run beside a recurrence), bias row sums fused.

    python tools/tools_wgrad_sweep.py          (GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import functional as Fn, _lib  # noqa: E402

R = 64 * 300
SHAPES = [("lstm 1024x256", 1024, 256), ("lin 256x256", 256, 256), ("kv 512x256", 512, 256),
          ("ffn 64x256", 64, 256), ("ffn 256x64", 256, 64)]


def timeit(fn, iters=20):
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
    dev = torch.device("cuda:0")
    for name, M, N in SHAPES:
        dY = torch.randn(R, M, device=dev)
        X = torch.randn(R, N, device=dev)
        C = torch.zeros(M, N, device=dev)
        gb = torch.zeros(M, device=dev)
        ref = dY.double().t() @ X.double()
        auto = Fn.wgrad_splits(M, N, R)
        line = [f"{name:14s} auto={auto:3d}"]
        for cap in (0, 1):
            prev = lib.mrg_gemm_set_blocks_per_cu(cap if cap < 2 else 0)
            pw = lib.mrg_gemm_set_glds_wg(1)
            for s in sorted({8, 16, 32, 64, 128, auto}):
                if s > R // 128:
                    continue

                def go():
                    Fn.gemm(M, N, R, Fn._ptr(dY), 1, M, Fn._ptr(X), 0, N, Fn._ptr(C), N, splits=s, device=dev,
                            asum_out=Fn._ptr(gb), asum_beta=0.0)
                us = timeit(go)
                err = ((C.double() - ref).abs().max() / ref.abs().max()).item()
                line.append(f"cap{cap}/s{s} {us:6.1f}us {2.0 * M * N * R / us / 1e6:4.0f}TF{'' if err < 1e-5 else ' ERR'}")
            lib.mrg_gemm_set_blocks_per_cu(prev)
            lib.mrg_gemm_set_glds_wg(pw)
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
