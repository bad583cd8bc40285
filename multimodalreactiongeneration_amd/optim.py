"""Fused AdamW over one flat parameter buffer (one libmrg launch per step).

Stands in for ``torch.optim.AdamW(self.parameters(), lr, weight_decay)`` of
``configure_optimizers`` (lstmformer.py:327-333, lstm_with_sample.py:248-254,
simple_lstm.py:193-199).  On construction every parameter is re-pointed into a
contiguous fp32 buffer and its ``.grad`` into a twin gradient buffer, so
``step()`` is a single kernel, ``zero_grad()`` a single memset and the DDP
reducer (``ddp.GradReducer``) all-reduces the gradient buffer in place.
It subclasses ``torch.optim.Optimizer`` so torch LR schedulers
(CosineAnnealingLR) drive ``param_groups[0]['lr']``.
"""
from __future__ import annotations

from typing import Iterable

import torch

from . import _lib
from .functional import _ptr, _stream


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

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        if g["lr"] != self._lr_on_device:  # LR scheduler moved it (once per epoch)
            self.step_lr[1].fill_(float(g["lr"]))
            self._lr_on_device = float(g["lr"])
        b1, b2 = g["betas"]
        _lib.check(_lib.load().mrg_adamw_step(
            _ptr(self.flat), _ptr(self.flat_grad), _ptr(self.exp_avg), _ptr(self.exp_avg_sq),
            self.flat.numel(), _ptr(self.step_lr), float(g["weight_decay"]), float(b1), float(b2),
            float(g["eps"]), _stream()), "adamw")
        return loss

    def zero_grad(self, set_to_none: bool = False):
        # gradients stay views of the flat buffer (set_to_none would detach them from it)
        self.flat_grad.zero_()
