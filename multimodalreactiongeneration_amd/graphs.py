"""HIP-graph capture of a whole training step.

Every op on the path is a fixed-shape HIP launch that neither allocates per call outside
torch's caching allocator nor synchronises with the host, so fwd + bwd (+ AdamW) of one step
can be recorded once and replayed: the per-launch host cost (Python, autograd, ctypes, the
HIP dispatch) is paid at capture only.  The scheduled-sampling decode of lstm_with_sampling
(lstm_with_sample.py:379-433) issues ~20k launches per step, so its step time is host-bound
without this.  Inputs must live in static device buffers that the caller refreshes in place
between replays (``buf.copy_(new)``).
"""
from typing import Callable, Sequence

import torch


def capture(step: Callable[[], object], warmup: int = 2, preserve: Sequence[torch.Tensor] = ()) -> Callable[[], None]:
    """Run ``step`` ``warmup`` times on a side stream (allocator and lazily created workspaces
    settle), record one call into a HIP graph and return its ``replay``.

    preserve: device tensors the warm-up must not change for good (e.g. ``opt.state_tensors()``
    when the step includes the optimizer): they are snapshotted first and restored after the
    capture, so the warm-up runs leave no update behind.  Recording itself executes nothing."""
    saved = [t.detach().clone() for t in preserve]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(max(1, warmup)):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    from . import functional as Fn
    Fn.reset_fork_point()
    try:
        with torch.cuda.graph(graph):
            step()
    finally:
        Fn.reset_fork_point()   # fork points are per capture (functional._fork's guard)
    with torch.no_grad():
        for t, v in zip(preserve, saved):
            t.copy_(v)
    torch.cuda.synchronize()
    return graph.replay
