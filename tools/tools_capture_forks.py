"""Does a HIP-graph capture keep a side stream's own ordering across repeated forks?

    python tools/tools_capture_forks.py        (GPU box)

main: x = 1; fork -> side: busy 20 ms, y = x + 1; fork again -> side: z = y + 1; join; main: w = z + 1.
Replayed: w must be 4.  Variants: a main-stream kernel between the forks or not.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import _lib  # noqa: E402


def run(between):
    lib = _lib.load()
    dev = torch.device("cuda:0")
    side = torch.cuda.Stream(device=dev)
    x = torch.zeros(1 << 20, device=dev)
    y, z, w = torch.zeros_like(x), torch.zeros_like(x), torch.zeros_like(x)
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(cap):
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cap):
            x.fill_(1.0)
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                lib.mrg_debug_busy(1, 64, 256, 20000.0, torch.cuda.current_stream().cuda_stream)
                torch.add(x, 1.0, out=y)
            if between:
                w.fill_(0.0)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                torch.add(y, 1.0, out=z)
            cur.wait_stream(side)
            torch.add(z, 1.0, out=w)
    for t in (x, y, z, w):
        t.fill_(-7.0)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    print(f"between={between}: x {x[0].item()} y {y[0].item()} z {z[0].item()} w {w[0].item()} (want 1 2 3 4)",
          flush=True)


if __name__ == "__main__":
    run(False)
    run(True)
