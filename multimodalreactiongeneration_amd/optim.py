"""Fused AdamW over one flat parameter buffer (one libmrg launch per step).

Stands in for ``torch.optim.AdamW(self.parameters(), lr, weight_decay)`` of
``configure_optimizers`` (lstmformer.py:327-333, lstm_with_sample.py:248-254,
simple_lstm.py:193-199).  On construction every parameter is re-pointed into a
contiguous fp32 buffer and its ``.grad`` into a twin gradient buffer, so
``step()`` is a single kernel, ``zero_grad()`` a single memset and the DDP
reducer (``ddp.GradReducer``) all-reduces the gradient buffer in place.
It subclasses ``torch.optim.Optimizer`` so torch LR schedulers
(CosineAnnealingLR) drive ``param_groups[0]['lr']``: the group is a dict whose
``'lr'`` assignment also writes the device-side LR the kernel reads, so a
scheduler stepped between HIP-graph replays takes effect in the replayed step.

Error surfacing: the persistent LSTM kernels OR a device flag on a hand-off
timeout; the AdamW kernel reads it and skips the update (garbage gradients never
reach the weights, replayed graphs included), and ``step()`` raises at the next
step once the flag, copied to pinned host memory without a sync, reads non-zero.
"""
from __future__ import annotations

from typing import Iterable

import torch

from . import _lib
from .functional import _ptr, _stream, _err_flag


def flatten_parameters(params, device=None):
    """Move parameters into one contiguous buffer; returns (flat_params, flat_grads, params)."""
    params = [p for p in params if p.requires_grad]
    if not params:
        raise ValueError("no trainable parameters")
    device = device or params[0].device
    n = sum(p.numel() for p in params)
    flat = torch.empty(n, dtype=torch.float32, device=device)
    gflat = torch.zeros(n, dtype=torch.float32, device=device)
    off = 0
    for p in params:
        k = p.numel()
        flat[off:off + k].copy_(p.detach().reshape(-1))
        p.data = flat[off:off + k].view_as(p)
        p.grad = gflat[off:off + k].view_as(p)
        off += k
    return flat, gflat, params


class _LRGroup(dict):
    """A param group whose 'lr' assignment (LR schedulers) is mirrored to the device buffer."""

    def __init__(self, group, opt):
        super().__init__(group)
        self._opt = opt

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        if k == "lr" and getattr(self, "_opt", None) is not None:
            self._opt._write_lr(v)


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params: Iterable, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        params = list(params)
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.flat, self.flat_grad, self.plist = flatten_parameters(params)
        dev = self.flat.device
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.step_lr = torch.tensor([0.0, float(lr)], dtype=torch.float32, device=dev)
        self._lr_on_device = float(lr)
        self._wrap_groups()
        self._err_host = self._err_event = None

    def _wrap_groups(self):
        self.param_groups[0] = _LRGroup(self.param_groups[0], self)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._wrap_groups()
        self._write_lr(self.param_groups[0]["lr"])

    def _write_lr(self, lr):
        lr = float(lr)
        if lr != self._lr_on_device:
            self.step_lr[1].fill_(lr)  # stream-ordered: lands before the next (replayed) step
            self._lr_on_device = lr

    def state_tensors(self):
        """Device state one update changes (graphs.capture(preserve=...) restores it after warm-up)."""
        return [self.flat, self.exp_avg, self.exp_avg_sq, self.step_lr]

    def _check_async(self):
        """Raise if an earlier step's persistent kernels reported a hand-off timeout (no sync: the
        flag is copied to pinned memory each step and read once that copy has completed)."""
        if not self.flat.is_cuda or torch.cuda.is_current_stream_capturing():
            return  # (no event queries inside a capture; replays are checked by check_errors())
        err = _err_flag(self.flat.device)
        if self._err_host is None:
            self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._err_event = torch.cuda.Event()
        elif self._err_event.query() and int(self._err_host[0]) != 0:
            self._err_host.zero_()
            err.zero_()
            raise RuntimeError("libmrg: LSTM recurrence hand-off timed out (grid not co-resident?); "
                               "the AdamW update of that step was skipped")
        self._err_host.copy_(err, non_blocking=True)
        self._err_event.record()

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        self._write_lr(g["lr"])
        self._check_async()
        b1, b2 = g["betas"]
        _lib.check(_lib.load().mrg_adamw_step(
            _ptr(self.flat), _ptr(self.flat_grad), _ptr(self.exp_avg), _ptr(self.exp_avg_sq),
            self.flat.numel(), _ptr(self.step_lr), float(g["weight_decay"]), float(b1), float(b2),
            float(g["eps"]), _ptr(_err_flag(self.flat.device)), _stream()), "adamw")
        from . import functional as Fn
        Fn.invalidate_weight_planes()  # the weights changed: their bf16 planes are stale
        return loss

    def zero_grad(self, set_to_none: bool = False):
        # gradients stay views of the flat buffer (set_to_none would detach them from it)
        if self.flat_grad.is_cuda:
            from . import functional as Fn
            Fn.zero_(self.flat_grad)
        else:
            self.flat_grad.zero_()
