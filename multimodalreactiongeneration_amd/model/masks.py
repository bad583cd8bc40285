"""Attention masks of the reference, kept symbolic.

gen_attention_mask (multi_modal_metaformer.py:32-79) materialises a bool
[B, heads, Tq, Tk] tensor (block-causal with ratio r, OR the AND of query and
key padding flags).  The MI355X kernels evaluate that rule from indices, so
here the mask is a small descriptor holding the two per-frame padding flag
vectors; ``dense()`` reproduces the reference tensor when one is needed.
"""
from __future__ import annotations

import torch

PADDING_VALUE = -100


class BlockCausalMask:
    """Descriptor equivalent to gen_attention_mask(main, other, heads, pad) (True = masked)."""

    def __init__(self, main_pad: torch.Tensor, other_pad: torch.Tensor, heads: int):
        self.main_pad = main_pad      # uint8 [B, Tq]
        self.other_pad = other_pad    # uint8 [B, Tk]
        self.heads = heads
        self.B, self.Tq = main_pad.shape
        self.Tk = other_pad.shape[1]

    # the reference reshapes the mask to [B*heads, Tq, Tk] before nn.MultiheadAttention
    def view(self, *shape):
        return self

    reshape = view

    @property
    def shape(self):
        return (self.B, self.heads, self.Tq, self.Tk)

    def dense(self) -> torch.Tensor:
        dev = self.main_pad.device
        i = torch.arange(self.Tq, device=dev).unsqueeze(1)
        j = torch.arange(self.Tk, device=dev).unsqueeze(0)
        if self.Tk % self.Tq == 0:
            causal = (j // (self.Tk // self.Tq)) > i
        else:
            causal = j > (i // (self.Tq // self.Tk))
        pad = self.main_pad.bool().unsqueeze(2) & self.other_pad.bool().unsqueeze(1)
        m = causal.unsqueeze(0) | pad
        return m.unsqueeze(1).expand(-1, self.heads, -1, -1)


def gen_attention_mask(main_modal: torch.Tensor, other_modal: torch.Tensor, head_num: int,
                       padding_value: float = PADDING_VALUE) -> BlockCausalMask:
    tq, tk = main_modal.shape[1], other_modal.shape[1]
    if tk % tq != 0 and tq % tk != 0:
        raise ValueError(f"other_modal_len must be divisible by main_modal_len. "
                         f"main_modal_len: {tq}, other_modal_len: {tk}")
    from .. import functional as Fn
    mp = Fn.padding_flags(main_modal, padding_value)
    op = mp if other_modal is main_modal else Fn.padding_flags(other_modal, padding_value)
    return BlockCausalMask(mp, op, head_num)
