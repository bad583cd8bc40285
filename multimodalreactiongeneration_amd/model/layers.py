"""Parameter-holding building blocks with the reference's module/parameter names.

Every class keeps the attribute names of the reference module it stands in
for, so ``state_dict`` keys and shapes are identical and reference checkpoints
load unchanged (model_loader.py:23-24).  All arithmetic is dispatched to
``functional`` (libmrg.so); there is no torch-math fallback.

  Linear, LayerNorm         nn.Linear / nn.LayerNorm holders
  LSTM                      nn.LSTM (weight_ih_l{k}[_reverse] ...)   -> functional.lstm_*
  MultiheadAttention        nn.MultiheadAttention (in_proj_*, out_proj) -> functional.mha
  ResidualConnection        residual_connection.py:5-37
  FeedForward               mixer_block.py:37-87
  LSTMSampler               lstm_sampler.py:6-34
  LSTMModule/LSTMBlock/LSTMLayerd   lstm_block.py:9-169
  MultiModalAttentionBlockSequential / MultimodalAttentionBlock / MultimodalAttention
                            multi_modal_att.py:6-91
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import List, Optional, Tuple

import torch
from torch import nn

from .. import functional as Fn
from .masks import BlockCausalMask

PADDING_VALUE = -100


def _unsupported(what):
    raise NotImplementedError(f"{what} is outside the MI355X path (SURVEY §2 scope)")


class Linear(nn.Linear):
    """nn.Linear whose forward runs the fp32 MFMA GEMM."""

    def forward(self, x):
        return Fn.linear(x, self.weight, self.bias)


class LayerNorm(nn.LayerNorm):
    def forward(self, x):  # standalone LayerNorm(x) == LN(x + 0)
        return Fn.residual_layernorm(x, torch.zeros_like(x), self.weight, self.bias, self.eps)


def make_activation(name):
    """set_nonlinearity (nonlinearity.py:6-16): 'relu' | 'swish' | 'tanh' | None/'none'."""
    if name is None or name == "none":
        return None
    if name == "relu":
        return nn.ReLU()
    if name == "swish":
        return nn.SiLU()
    if name == "tanh":
        return nn.Tanh()
    raise ValueError("nonlinearity must be in ['relu', 'swish', 'tanh', None]")


def run_sequential_ffn(seq: nn.Sequential, x):
    """Run an nn.Sequential of Linear [-> ReLU -> Linear] through the fused kernels."""
    mods = list(seq.children())
    if len(mods) == 1 and isinstance(mods[0], nn.Linear):
        return Fn.linear(x, mods[0].weight, mods[0].bias)
    if len(mods) == 3 and isinstance(mods[1], nn.ReLU):
        return Fn.ffn(x, mods[0].weight, mods[0].bias, mods[2].weight, mods[2].bias)
    if len(mods) == 2 and all(isinstance(m, nn.Linear) for m in mods):
        return Fn.linear(Fn.linear(x, mods[0].weight, mods[0].bias), mods[1].weight, mods[1].bias)
    _unsupported(f"feed-forward {[type(m).__name__ for m in mods]}")


class ResidualConnection(nn.Module):
    """LN(module(x, ...) + x); tuple outputs keep their tail (residual_connection.py:20-37)."""

    def __init__(self, module: nn.Module, use_layer_norm=True, num_nodes: int = -1, dropout=0.0):
        super().__init__()
        if use_layer_norm and num_nodes == -1:
            raise ValueError("num_nodes must be specified when use_layer_norm is set to True.")
        self.module = module
        self.use_layer_norm = use_layer_norm
        self.layer_norm = LayerNorm(num_nodes) if use_layer_norm else None
        self.dropout = nn.Dropout(dropout)
        if dropout:
            _unsupported("dropout > 0")

    def combine(self, y, x):
        if self.layer_norm is not None:
            return Fn.residual_layernorm(y, x, self.layer_norm.weight, self.layer_norm.bias,
                                         self.layer_norm.eps)
        _unsupported("residual without LayerNorm")

    def forward(self, x, *args, **kwargs):
        # modules that can run LN(module(x) + x) as one fused op (the residual branch's gradient is
        # added by their input-gradient GEMM) expose fused_residual_ln; None = not eligible here
        fused = getattr(self.module, "fused_residual_ln", None)
        if fused is not None and self.layer_norm is not None:
            out = fused(self.layer_norm, x, *args, **kwargs)
            if out is not None:
                return out
        y = self.module(x, *args, **kwargs)
        rest = None
        if isinstance(y, (tuple, list)):
            y, rest = y[0], tuple(y[1:])
        y = self.combine(y, x)
        return y if rest is None else (y, *rest)


class FeedForward(nn.Module):
    """Linear (nonlinearity none) or Linear->act->Linear, optional residual + LN (mixer_block.py:37-87)."""

    def __init__(self, hidden_size: int, bottleneck_size: int = None, output_size: int = None,
                 nonlinearity=None, residual: bool = False, residual_layer_norm: bool = False,
                 bias: bool = True, device=None, dtype=None):
        super().__init__()
        bottleneck_size = hidden_size if bottleneck_size is None else bottleneck_size
        output_size = hidden_size if output_size is None else output_size
        if hidden_size != output_size and residual:
            raise ValueError("hidden_size must be equal to output_size when residual is True.")
        act = make_activation(nonlinearity)
        if act is None:
            arch = OrderedDict([("feedforward", Linear(hidden_size, output_size, bias=bias))])
        else:
            arch = OrderedDict([("input", Linear(hidden_size, bottleneck_size, bias=bias)),
                                ("activation", act),
                                ("output", Linear(bottleneck_size, output_size, bias=bias))])
        self.feed_forward = nn.Sequential(arch)
        if residual:
            self.feed_forward = ResidualConnection(self.feed_forward, residual_layer_norm, hidden_size)

    def forward(self, x):
        ff = self.feed_forward
        if isinstance(ff, ResidualConnection):
            ln = ff.layer_norm
            mods = list(ff.module.children())
            if ln is not None and len(mods) == 1 and isinstance(mods[0], nn.Linear):
                return Fn.linear_residual_layernorm(x, mods[0].weight, mods[0].bias, ln.weight, ln.bias, ln.eps)
            if ln is not None and len(mods) == 3 and isinstance(mods[1], nn.ReLU):
                return Fn.ffn_residual_layernorm(x, mods[0].weight, mods[0].bias, mods[2].weight, mods[2].bias,
                                                 ln.weight, ln.bias, ln.eps)
            return ff.combine(run_sequential_ffn(ff.module, x), x)
        return run_sequential_ffn(ff, x)


class LSTM(nn.Module):
    """nn.LSTM parameter layout (batch_first) running the persistent HIP recurrence."""

    def __init__(self, input_size, hidden_size, num_layers=1, bias=True, batch_first=True,
                 dropout=0.0, bidirectional=False, proj_size=0, device=None, dtype=None):
        super().__init__()
        if proj_size:
            _unsupported("LSTM proj_size")
        if not batch_first:
            _unsupported("LSTM batch_first=False")
        if not bias:
            _unsupported("LSTM without bias")
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.bidirectional, self.dropout, self.batch_first = bidirectional, dropout, batch_first
        D = 2 if bidirectional else 1
        k = 1.0 / math.sqrt(hidden_size)
        for layer in range(num_layers):
            in_sz = input_size if layer == 0 else hidden_size * D
            for d in range(D):
                sfx = f"l{layer}" + ("_reverse" if d else "")
                for name, shape in ((f"weight_ih_{sfx}", (4 * hidden_size, in_sz)),
                                    (f"weight_hh_{sfx}", (4 * hidden_size, hidden_size)),
                                    (f"bias_ih_{sfx}", (4 * hidden_size,)),
                                    (f"bias_hh_{sfx}", (4 * hidden_size,))):
                    p = nn.Parameter(torch.empty(shape, device=device, dtype=dtype))
                    nn.init.uniform_(p, -k, k)
                    self.register_parameter(name, p)

    def direction_params(self, layer, reverse=False):
        sfx = f"l{layer}" + ("_reverse" if reverse else "")
        return (getattr(self, f"weight_ih_{sfx}"), getattr(self, f"weight_hh_{sfx}"),
                getattr(self, f"bias_ih_{sfx}"), getattr(self, f"bias_hh_{sfx}"))

    def forward(self, x, hx=None):
        pre = self.__dict__.pop("_paired_out", None)   # computed in a shared launch (paired_lstm_layerd)
        if pre is not None:
            if pre[0] is not x:
                raise RuntimeError("LSTM: a paired result was left for a different input")
            return pre[1]
        if self.dropout and self.training and self.num_layers > 1:
            _unsupported("LSTM inter-layer dropout")
        D = 2 if self.bidirectional else 1
        hs, cs = [], []
        for layer in range(self.num_layers):
            if D == 1:
                h0 = None if hx is None else hx[0][layer]
                c0 = None if hx is None else hx[1][layer]
                x, hT, cT = Fn.lstm_layer(x, *self.direction_params(layer), h0, c0)
                hs.append(hT)
                cs.append(cT)
            else:
                h0 = None if hx is None else hx[0][2 * layer:2 * layer + 2]
                c0 = None if hx is None else hx[1][2 * layer:2 * layer + 2]
                x, hT, cT = Fn.lstm_bidirectional_layer(x, self.direction_params(layer, False),
                                                        self.direction_params(layer, True), h0, c0)
                hs += [hT[0], hT[1]]
                cs += [cT[0], cT[1]]
        if len(hs) == 1:  # one layer, one direction: a view, no copy kernel (T = 1 decode frames)
            return x, (hs[0].unsqueeze(0), cs[0].unsqueeze(0))
        return x, (torch.stack(hs), torch.stack(cs))


class GRU(nn.Module):
    """nn.GRU parameter layout (batch_first; gate order r, z, n) on the GRU cell kernels."""

    def __init__(self, input_size, hidden_size, num_layers=1, bias=True, batch_first=True,
                 dropout=0.0, bidirectional=False, device=None, dtype=None):
        super().__init__()
        if not batch_first:
            _unsupported("GRU batch_first=False")
        if not bias:
            _unsupported("GRU without bias")
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.bidirectional, self.dropout, self.batch_first = bidirectional, dropout, batch_first
        D = 2 if bidirectional else 1
        k = 1.0 / math.sqrt(hidden_size)
        for layer in range(num_layers):
            in_sz = input_size if layer == 0 else hidden_size * D
            for d in range(D):
                sfx = f"l{layer}" + ("_reverse" if d else "")
                for name, shape in ((f"weight_ih_{sfx}", (3 * hidden_size, in_sz)),
                                    (f"weight_hh_{sfx}", (3 * hidden_size, hidden_size)),
                                    (f"bias_ih_{sfx}", (3 * hidden_size,)),
                                    (f"bias_hh_{sfx}", (3 * hidden_size,))):
                    p = nn.Parameter(torch.empty(shape, device=device, dtype=dtype))
                    nn.init.uniform_(p, -k, k)
                    self.register_parameter(name, p)

    def direction_params(self, layer, reverse=False):
        sfx = f"l{layer}" + ("_reverse" if reverse else "")
        return (getattr(self, f"weight_ih_{sfx}"), getattr(self, f"weight_hh_{sfx}"),
                getattr(self, f"bias_ih_{sfx}"), getattr(self, f"bias_hh_{sfx}"))

    def forward(self, x, hx=None):
        if self.dropout and self.training and self.num_layers > 1:
            _unsupported("GRU inter-layer dropout")
        D = 2 if self.bidirectional else 1
        hs = []
        for layer in range(self.num_layers):
            ys = []
            for d in range(D):
                h0 = None if hx is None else hx[layer * D + d]
                y, hT = Fn.gru_layer(x, *self.direction_params(layer, bool(d)), h0, reverse=bool(d))
                ys.append(y)
                hs.append(hT)
            x = ys[0] if D == 1 else torch.cat(ys, dim=-1)
        return x, torch.stack(hs)


class MultiheadAttention(nn.Module):
    """nn.MultiheadAttention parameter layout (kdim = vdim = embed_dim, batch_first)."""

    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=True, add_bias_kv=False,
                 add_zero_attn=False, kdim=None, vdim=None, batch_first=False, device=None, dtype=None):
        super().__init__()
        if add_bias_kv or add_zero_attn:
            _unsupported("MHA add_bias_kv / add_zero_attn")
        if (kdim not in (None, embed_dim)) or (vdim not in (None, embed_dim)):
            _unsupported("MHA kdim/vdim != embed_dim")
        if not bias:
            _unsupported("MHA without bias")
        if embed_dim % num_heads:
            raise AssertionError("embed_dim must be divisible by num_heads")
        self.embed_dim, self.num_heads, self.dropout, self.batch_first = embed_dim, num_heads, dropout, batch_first
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim, device=device, dtype=dtype))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * embed_dim, device=device, dtype=dtype))
        self.out_proj = Linear(embed_dim, embed_dim, bias=True, device=device, dtype=dtype)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)

    def forward(self, query, key, value, key_padding_mask=None, need_weights=False, attn_mask=None,
                average_attn_weights=False, is_causal=False):
        if key is not value:
            _unsupported("MHA with distinct key and value tensors")
        if key_padding_mask is not None or need_weights:
            _unsupported("MHA key_padding_mask / need_weights")
        if self.dropout and self.training:
            _unsupported("attention dropout")
        if not self.batch_first:
            query, key = query.transpose(0, 1), key.transpose(0, 1)
        causal, qpad, kpad = False, None, None
        if attn_mask is not None:
            if not isinstance(attn_mask, BlockCausalMask):
                _unsupported("dense attn_mask (use masks.gen_attention_mask)")
            causal, qpad, kpad = True, attn_mask.main_pad, attn_mask.other_pad
        out = Fn.mha(query, key, self.in_proj_weight, self.in_proj_bias, self.out_proj.weight,
                     self.out_proj.bias, self.num_heads, causal, qpad, kpad)
        if not self.batch_first:
            out = out.transpose(0, 1)
        return out, None


class MHAforSequentail(nn.Module):
    """(q, k, v, kpm, need_weights, attn_mask, avg, is_causal) tuple interface (for_sequential.py:8-51)."""

    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=True, add_bias_kv=False,
                 add_zero_attn=False, kdim=None, vdim=None, batch_first=False, nonlinearity=None,
                 device=None, dtype=None):
        super().__init__()
        self.mha = MultiheadAttention(embed_dim, num_heads, dropout, bias, add_bias_kv, add_zero_attn,
                                      kdim, vdim, batch_first, device=device, dtype=dtype)
        self.nonlinearity = make_activation(nonlinearity)
        if self.nonlinearity is not None:
            _unsupported("MHA output nonlinearity (reference Q7 path)")

    def forward(self, x):
        x = list(x)
        x[4] = False
        x[6] = False
        return self.mha(*x)


class LSTMSampler(nn.Module):
    """LSTM over the audio frames keeping every r-th output (lstm_sampler.py:6-34)."""

    def __init__(self, hiddn_size: int, num_layers: int, dropout: float, decline_rate: int,
                 bidirectional=False):
        super().__init__()
        self.sampler = LSTM(hiddn_size, hiddn_size, num_layers=num_layers, dropout=dropout,
                            bidirectional=bidirectional, batch_first=True)
        self.decline_rate = decline_rate

    def forward(self, x, hx=None):
        h, hx = self.sampler(x, hx)
        r = self.decline_rate
        return h[:, r - 1::r, :].contiguous(), hx


class LSTMModule(nn.Module):
    """nn.LSTM [+ mixing Linear] (lstm_block.py:9-46)."""

    def __init__(self, input_size=256, hidden_size=128, num_layers=1, output_size=256, dropout=0.0,
                 bidirectional=True, use_mixing=True):
        super().__init__()
        self.lstm_module = LSTM(input_size, hidden_size, num_layers=num_layers, dropout=dropout,
                                batch_first=True, bidirectional=bidirectional)
        out = hidden_size * (2 if bidirectional else 1)
        self.mixer = Linear(out, output_size) if use_mixing else None
        if not use_mixing and out != output_size:
            raise ValueError("lstm_out_size must be equal to output_size when use_mixing is False.")

    def forward(self, input_tensor, hx=None):
        hs, hx = self.lstm_module(input_tensor, hx)
        y = hs if self.mixer is None else self.mixer(hs)
        return y, hx


class LSTMBlock(nn.Module):
    """Residual LSTMModule [+ residual FFN] (lstm_block.py:49-103)."""

    def __init__(self, input_size=256, hidden_size=128, lstm_out_size=256, num_layers=1,
                 bottleneck_size=64, output_size=256, dropout=0.0, bidirectional=True,
                 use_layer_norm=True, use_relu=True, use_mixing=False, use_residual=True,
                 use_feed_forward=True):
        super().__init__()
        if use_residual and input_size != lstm_out_size or lstm_out_size != output_size:
            raise ValueError("input_size must be equal to lstm_out_size and output_size when use_residuals.")
        self.use_feed_forward = use_feed_forward
        self.lstm_module = LSTMModule(input_size, hidden_size, num_layers, lstm_out_size, dropout,
                                      bidirectional, use_mixing)
        if use_feed_forward:
            seq = OrderedDict()
            seq["input"] = Linear(lstm_out_size, bottleneck_size)
            if use_relu:
                seq["relu"] = nn.ReLU()
            seq["mapping"] = Linear(bottleneck_size, output_size)
            self.feed_forward_module = nn.Sequential(seq)
        if use_residual:
            self.lstm_module = ResidualConnection(self.lstm_module, use_layer_norm, lstm_out_size, dropout)
            if use_feed_forward:
                self.feed_forward_module = ResidualConnection(self.feed_forward_module, use_layer_norm,
                                                              output_size, dropout)

    def forward(self, input_tenor, hx=None):
        y, hx = self.lstm_module(input_tenor, hx)
        if self.use_feed_forward:
            ff = self.feed_forward_module
            if isinstance(ff, ResidualConnection):
                y = ff.combine(run_sequential_ffn(ff.module, y), y)
            else:
                y = run_sequential_ffn(ff, y)
        return y, hx


class LSTMLayerd(nn.Module):
    """Stack of LSTMBlocks; returns the INPUT hxs (reference quirk Q2, lstm_block.py:169)."""

    def __init__(self, input_size=256, lstm_hidden_size=128, affine_hidden_size=256, bottleneck_size=64,
                 num_layers=2, num_layers_per_block=1, output_size=256, dropout=0.0, bidirectional=True,
                 use_layer_norm=True, use_relu=True, use_mixing=False, use_residual=True,
                 use_feed_forward=True):
        super().__init__()
        D = 2 if bidirectional else 1
        lstm_out = lstm_hidden_size * D
        affine = affine_hidden_size if use_mixing else lstm_out
        self.lstm_layered = nn.ModuleList()
        for i in range(num_layers):
            self.lstm_layered.append(LSTMBlock(
                input_size=input_size if i == 0 else affine, hidden_size=lstm_hidden_size,
                lstm_out_size=affine, num_layers=num_layers_per_block, bottleneck_size=bottleneck_size,
                output_size=output_size if i == num_layers - 1 else affine, dropout=dropout,
                bidirectional=bidirectional, use_layer_norm=use_layer_norm, use_relu=use_relu,
                use_mixing=use_mixing, use_residual=use_residual, use_feed_forward=use_feed_forward))

    def forward(self, input_tensor, hxs=None):
        for i, block in enumerate(self.lstm_layered):
            input_tensor, _ = block(input_tensor, None if hxs is None else hxs[i])
        return input_tensor, hxs


def _block_lstm(block):
    """The LSTM inside an LSTMBlock (through its ResidualConnection and LSTMModule), or None."""
    m = block.lstm_module
    m = getattr(m, "module", m)
    lstm = getattr(m, "lstm_module", None)
    return lstm if isinstance(lstm, LSTM) else None


def paired_lstm_layerd(stacks, xs):
    """Independent LSTMLayerd stacks over their own inputs (SimpleLSTM's acoustic and motion encoders,
    simple_lstm.py:146-207) with block i's bidirectional recurrences of ALL stacks in one persistent
    launch (functional.lstm_bidirectional_layers), the rest of each block as usual.  Returns the
    stacks' outputs, or None when they are outside that form (different depth, hidden size, B or T,
    multi-layer LSTMs, one direction)."""
    nb = len(stacks[0].lstm_layered)
    if any(len(st.lstm_layered) != nb for st in stacks) or len({tuple(x.shape[:2]) for x in xs}) != 1:
        return None
    lstms = [[_block_lstm(b) for b in st.lstm_layered] for st in stacks]
    for col in zip(*lstms):
        if any(l is None or l.num_layers != 1 or not l.bidirectional for l in col):
            return None
        if len({l.hidden_size for l in col}) != 1:
            return None
    xs = list(xs)
    for i in range(nb):
        res = Fn.lstm_bidirectional_layers([(x, ls[i].direction_params(0, False), ls[i].direction_params(0, True))
                                            for x, ls in zip(xs, lstms)])
        for k, (st, ls) in enumerate(zip(stacks, lstms)):
            y, hT, cT = res[k]
            ls[i]._paired_out = (xs[k], (y, (hT, cT)))
            try:
                xs[k], _ = st.lstm_layered[i](xs[k], None)
            finally:
                ls[i].__dict__.pop("_paired_out", None)
    return xs


class MultiModalAttentionBlockSequential(nn.Module):
    """Unmasked cross-attention + projection (multi_modal_att.py:6-31)."""

    def __init__(self, modal1_feat_size=256, modal2_feat_size=256, num_head=1, dropout=0.0):
        super().__init__()
        self.cross_modal_att = MultiheadAttention(modal1_feat_size, num_head, dropout=dropout,
                                                  batch_first=True, kdim=modal2_feat_size,
                                                  vdim=modal2_feat_size)
        self.projection = Linear(modal1_feat_size, modal1_feat_size)

    def forward(self, modal1, modal2):
        o, _ = self.cross_modal_att(modal1, modal2, modal2)
        return self.projection(o)


class MultimodalAttentionBlock(nn.Module):
    def __init__(self, modal1_feat_size=256, modal2_feat_size=256, num_head=1, dropout=0.0,
                 use_residual=True, use_layer_norm=True):
        super().__init__()
        self.att_module = MultiModalAttentionBlockSequential(modal1_feat_size, modal2_feat_size,
                                                             num_head, dropout)
        if use_residual:
            self.att_module = ResidualConnection(self.att_module, use_layer_norm, modal1_feat_size)

    def forward(self, modal1, modal2):
        return self.att_module(modal1, modal2)


class MultimodalAttention(nn.Module):
    def __init__(self, modal1_feat_size=256, modal2_feat_size=256, num_head=1, num_layers=1,
                 dropout=0.0, use_residual=True, use_layer_norm=True):
        super().__init__()
        self.att_layers = nn.ModuleList([
            MultimodalAttentionBlock(modal1_feat_size, modal2_feat_size, num_head, dropout,
                                     use_residual, use_layer_norm) for _ in range(num_layers)])

    def forward(self, modal1, modal2):
        for layer in self.att_layers:
            modal1 = layer(modal1, modal2)
        return modal1
