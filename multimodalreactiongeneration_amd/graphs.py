"""HIP-graph capture of a whole training step.

Every op on the path is a fixed-shape HIP launch that neither allocates per call outside
torch's caching allocator nor synchronises with the host, so fwd + bwd (+ AdamW) of one step
can be recorded once and replayed: the per-launch host cost (Python, autograd, ctypes, the
HIP dispatch) is paid at capture only.  The scheduled-sampling decode of lstm_with_sampling
(lstm_with_sample.py:379-433) issues ~20k launches per step, so its step time is host-bound
without this.  Inputs must live in static device buffers that the caller refreshes in place
between replays (``buf.copy_(new)``).
"""
from typing import Callable

import torch


def capture(step: Callable[[], object], warmup: int = 2) -> Callable[[], None]:
    """Run ``step`` ``warmup`` times on a side stream (allocator and lazily created workspaces
    settle), record one call into a HIP graph and return its ``replay``."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(max(1, warmup)):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    return graph.replay
