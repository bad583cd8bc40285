"""Data-parallel gradient all-reduce over RCCL (torch.distributed backend "nccl" == RCCL on ROCm).

Reference: Lightning ``strategy: ddp`` (mr_gen/model/lstmformer/config.yaml:127)
= one process per GPU, gradients averaged across ranks after backward.  Here
the gradients already live in ONE flat fp32 buffer (optim.FusedAdamW), so the
exchange is a single in-place all-reduce (ReduceOp.AVG) of 52.2 MB for the
benchmark model, issued on a dedicated communication stream so it can be
overlapped with other work; the optimizer stream waits on it.  With the gloo
backend (CPU tests) AVG is emulated by SUM then a scale.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*); no-op at world 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 or dist.is_initialized():
        return dist.get_rank() if dist.is_initialized() else 0, world
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


def broadcast_parameters(module: torch.nn.Module, src: int = 0):
    """Same initial weights on every rank (DDP does this at wrap time)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return
    with torch.no_grad():
        for p in module.parameters():
            dist.broadcast(p.data, src)


class GradReducer:
    """Average a flat gradient buffer across ranks, in buckets, on a side stream."""

    def __init__(self, flat_grad: torch.Tensor, bucket_elems: int = 0):
        self.flat_grad = flat_grad
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.backend = dist.get_backend() if dist.is_initialized() else None
        n = flat_grad.numel()
        if bucket_elems <= 0:
            bucket_elems = n
        self.buckets = [(s, min(n, s + bucket_elems)) for s in range(0, n, bucket_elems)]
        self.stream = torch.cuda.Stream(device=flat_grad.device) if flat_grad.is_cuda else None

    def allreduce(self):
        if self.world <= 1:
            return
        use_avg = self.backend == "nccl"
        op = dist.ReduceOp.AVG if use_avg else dist.ReduceOp.SUM
        if self.stream is not None:
            cur = torch.cuda.current_stream(self.flat_grad.device)
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                for s, e in self.buckets:
                    dist.all_reduce(self.flat_grad[s:e], op=op)
            cur.wait_stream(self.stream)
        else:
            for s, e in self.buckets:
                dist.all_reduce(self.flat_grad[s:e], op=op)
        if not use_avg:
            self.flat_grad.mul_(1.0 / self.world)
