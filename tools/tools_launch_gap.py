"""What one kernel boundary costs on the critical path: N dependent tiny kernels on one stream, eager
and as one replayed HIP graph, and the same with 256-workgroup kernels (so the dispatch has to fill
the chip), reported as microseconds per kernel.

    python tools/tools_launch_gap.py         (GPU box)
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402


def per_kernel_us(fn, n, reps=5):
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best / n * 1e6


def main():
    dev = torch.device("cuda:0")
    n = 400
    for nbytes in (1024, 4 << 20):   # one workgroup / many workgroups per fill
        buf = torch.empty(nbytes // 4, device=dev)

        def chain():
            for _ in range(n):
                Fn.zero_(buf)
        chain()
        eager = per_kernel_us(chain, n)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            chain()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                chain()
        graph = per_kernel_us(g.replay, n)
        print(f"fill of {nbytes} B x {n} dependent launches: eager {eager:.2f} us/kernel, "
              f"graph replay {graph:.2f} us/kernel", flush=True)


if __name__ == "__main__":
    main()
