"""One weight-gradient product shape of the step (dW += dY^T X, 19200 x 1024 x 256, the fused bias sums),
REPS times, for counter passes (rocprofv3 --pmc ... -- python3 tools/wgrad_one.py).

    python tools/wgrad_one.py [REPS]       (GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402


def main(reps):
    dev = torch.device("cuda", 0)
    Fn.set_wgrad_stream(False)
    rows, N, In = 19200, 1024, 256
    dy, x = torch.randn(rows, N, device=dev), torch.randn(rows, In, device=dev)
    gw, gb = torch.zeros(N, In, device=dev), torch.zeros(N, device=dev)
    f = lambda: Fn._wgrad(Fn._ptr(dy), N, Fn._ptr(x), In, rows, N, In, gw, dev, gb=gb)  # noqa: E731
    f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"{rows}x{N}x{In} splits {Fn.wgrad_splits(N, In, rows)}: {us:.1f} us per product "
          f"({2.0 * rows * N * In / us / 1e6:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
